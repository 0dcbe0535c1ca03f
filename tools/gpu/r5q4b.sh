set -o pipefail
# final Q4_0 build: the Q4_0 / Q8_0 GPU tests, the 32-row gate/up, then the prefill PMC breakdown
O=gpurun_out/r5q4b; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_q4_0_gpu.py tests/test_q8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for q in q4_0 q8_0; do timeout -k 10 200 python -u tools/step_probe.py --M 32 --kinds 2 --quant $q; done || exit 1
bash tools/gpu/r5pmc_prefill.sh
