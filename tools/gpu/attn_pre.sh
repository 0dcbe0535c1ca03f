# attention: first K/V chunk issued with q; parity tests then batch-1 timing (graph replay)
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "decode_steps or persistent or batch_greedy or prefill_logits" > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/attn_tests.log
for i in 1 2 3; do
  echo "now $(timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1)"
done
