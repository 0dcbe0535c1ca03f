set -o pipefail
# in-work-group K halves (MX_KQ_KH2 / MX_Q8_KH2) for the 32-row quantised gate/up: parity, then A/B
O=gpurun_out/r5kh2; mkdir -p $O
export MX_KQ_KH2=1 MX_Q8_KH2=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kquants_gpu.py -k "wide" tests/test_q4_0_gpu.py -k "wide" tests/test_q8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
unset MX_KQ_KH2 MX_Q8_KH2
for r in 1 2; do
for q in q4_0 q8_0 q4_k_m; do
timeout -k 10 200 python -u tools/step_probe.py --M 32 --kinds 2 --quant $q > $O/a_${q}_$r.json || exit 1
MX_KQ_KH2=1 MX_Q8_KH2=1 timeout -k 10 200 python -u tools/step_probe.py --M 32 --kinds 2 --quant $q > $O/b_${q}_$r.json || exit 1
done; done
for f in $O/*.json; do echo "$f $(cat $f)"; done
