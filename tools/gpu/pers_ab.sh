# row-tile-persistent gate/up: parity tests, then interleaved batch-1 A/B (graph replay)
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "persistent_gate_up or decode_steps" > gpurun_out/pers_tests.log 2>&1 || { tail -40 gpurun_out/pers_tests.log; exit 1; }
grep -E "PASS|FAIL|max\|d\|" gpurun_out/pers_tests.log | tail -12
for i in 1 2; do
  echo "base $(MX_NO_PERS=1 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
  echo "pers $(timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
  echo "pers_u8 $(MX_PERS_U=8 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
done
