# phantom-tile persistent GEMVs (TinyLlama gate/up, lm_head with norm on load): parity, then A/B
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "decode_steps or persistent or batch_greedy or prefill_logits or 70b_geometry" > gpurun_out/p4_tests.log 2>&1 || { tail -40 gpurun_out/p4_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/p4_tests.log
for i in 1 2; do
  for m in tinyllama-1.1b llama3-8b; do
    echo "$m base $(MX_NO_PERS=1 timeout -k 10 120 python3 tools/q8_decode.py --model $m --bf16 --rows 1)"
    echo "$m nohead $(MX_NO_PERS_HEAD=1 timeout -k 10 120 python3 tools/q8_decode.py --model $m --bf16 --rows 1)"
    echo "$m pers $(timeout -k 10 120 python3 tools/q8_decode.py --model $m --bf16 --rows 1)"
  done
done
