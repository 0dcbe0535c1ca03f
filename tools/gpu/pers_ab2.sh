# row-tile-persistent GEMVs: batch-1 A/B (graph replay), interleaved; then parity with the RESID variant on
export TMPDIR=/tmp
set -e
for i in 1 2; do
  echo "base     $(MX_NO_PERS=1 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
  echo "u8       $(timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
  echo "u16      $(MX_PERS_U=16 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
  echo "u8+resid $(MX_PERS_RESID=1 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
done
MX_PERS_RESID=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "persistent_gate_up or decode_steps" > gpurun_out/pers_tests.log 2>&1 || { tail -40 gpurun_out/pers_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pers_tests.log | tail -8
