# A/B: one-token Q8_0 / Q4_0 gate/up as a tile-walking group with one quantised image (MX_Q8_PERS_QL)
# (record of the A/B: MX_Q8_PERS_QL became the default afterwards; MX_NO_Q8_PERS_QL=1 now selects the old form)
set -o pipefail
O=gpurun_out/r5pql; mkdir -p $O
MX_Q8_PERS_QL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_q8_gpu.py tests/test_q4_0_gpu.py > $O/p.log 2>&1 || { tail -30 $O/p.log; exit 1; }
echo "parity with MX_Q8_PERS_QL: $(tail -1 $O/p.log)"
for r in 1 2; do for v in base pers; do
  if [ $v = pers ]; then export MX_Q8_PERS_QL=1; else unset MX_Q8_PERS_QL; fi
  timeout -k 10 200 python -u tools/step_probe.py --quant q4_0 --M 1 --kinds 2 > $O/s4$v$r.log 2>&1 || { tail -20 $O/s4$v$r.log; exit 1; }
  timeout -k 10 200 python -u tools/step_probe.py --quant q8_0 --M 1 --kinds 2 > $O/s8$v$r.log 2>&1 || { tail -20 $O/s8$v$r.log; exit 1; }
  timeout -k 10 300 python -u tools/quant_step.py q4_0 q8_0 > $O/q$v$r.log 2>&1 || { tail -20 $O/q$v$r.log; exit 1; }
  echo "$v run $r q4_0 $(grep -o '"gate_up": {[^}]*}' $O/s4$v$r.log) q8_0 $(grep -o '"gate_up": {[^}]*}' $O/s8$v$r.log)"
  grep wtype $O/q$v$r.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('   $v', d['wtype'], 'batch1', d['batch1']['ms_per_token'], 'M32', d['decode']['ms_per_step'])"
done; done
