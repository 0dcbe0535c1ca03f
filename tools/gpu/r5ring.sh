set -o pipefail
# wide GEMV weight ring 4 chunks (MX_WIDE_RING=4) vs 2: 32-row parity tests, per-kernel probe, bench A/B
O=gpurun_out/r5ring; mkdir -p $O
MX_WIDE_RING=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_baseline_gpu.py tests/test_gpu_sharing_gpu.py tests/test_engine_gpu.py tests/test_fulldepth_stages_gpu.py -k "not config5" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 2 4; do MX_WIDE_RING=$v timeout -k 10 200 python -u tools/step_probe.py --M 32 --kinds 0,1,2,3,4 > $O/probe_$v.json || exit 1; cat $O/probe_$v.json; done
bash tools/gpu/ab_env.sh r5ring/ab "MX_WIDE_RING=2 MX_WIDE_RING=4" "--steps 64 --warmup 8"
