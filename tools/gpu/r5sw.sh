set -o pipefail
# swapped-operand Q8_0 / Q4_0 32-row gate/up (MX_Q8_SWAP=1: one K set, 2: two K sets): parity, then A/B
O=gpurun_out/r5sw; mkdir -p $O
for v in 1 2; do
MX_Q8_SWAP=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_q4_0_gpu.py tests/test_q8_gpu.py -k "wide or loop" > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
for r in 1 2; do
for q in q4_0 q8_0; do
for v in 0 1 2; do
MX_Q8_SWAP=$v timeout -k 10 200 python -u tools/step_probe.py --M 32 --kinds 2 --quant $q > $O/${q}_sw${v}_$r.json || exit 1
done; done; done
for f in $O/*.json; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(d['gate_up'])")"; done
