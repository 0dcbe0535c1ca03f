# TinyLlama attn_output / ffn_down as split-K (2 groups per tile, in-launch fold): parity, then A/B
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "decode_steps or persistent or batch_greedy" > gpurun_out/kz_tests.log 2>&1 || { tail -40 gpurun_out/kz_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/kz_tests.log
for i in 1 2 3; do
  echo "noresid $(MX_NO_PERS_RESID=1 timeout -k 10 120 python3 tools/q8_decode.py --model tinyllama-1.1b --bf16 --rows 1)"
  echo "kz      $(timeout -k 10 120 python3 tools/q8_decode.py --model tinyllama-1.1b --bf16 --rows 1)"
done
echo "8b      $(timeout -k 10 120 python3 tools/q8_decode.py --model llama3-8b --bf16 --rows 1)"
