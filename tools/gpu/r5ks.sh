set -o pipefail
# split-K targets of the 32-row slab GEMVs (MX_WIDE_KS=q|k|v,attn_output,ffn_down): bench main line, interleaved
O=gpurun_out/r5ks; mkdir -p $O
MX_WIDE_KS=2,2,4 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_baseline_gpu.py tests/test_gpu_sharing_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/ab_env.sh r5ks/ab "- MX_WIDE_KS=2,4,8 MX_WIDE_KS=4,2,8 MX_WIDE_KS=4,4,4 MX_WIDE_KS=2,2,4" "--steps 64 --warmup 8 --batch1-steps 0 --tiny-tokens 0 --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --serve-requests 0 --geometry-steps 0"
