# one-token split-K qkv: parity tests, then interleaved batch-1 A/B (graph replay)
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "decode_steps or persistent or batch_greedy or 70b_geometry or submit_wait or long_context" > gpurun_out/qs_tests.log 2>&1 || { tail -40 gpurun_out/qs_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/qs_tests.log
for i in 1 2 3; do
  echo "nosplit $(MX_NO_QKV_SPLIT=1 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1)"
  echo "split   $(timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1)"
done
