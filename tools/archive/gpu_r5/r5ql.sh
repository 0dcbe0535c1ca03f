# batch-1 Q8_0 / Q4_0: gate/up quantising its operand on load (product) vs a norm + quantise launch
# (MX_Q8_GU_NOQL); whole steps (tools/quant_step.py) and per-kernel times in both forms
# (record of a finished A/B: the switch it sets was removed from the engine afterwards -- see git log for the build it ran on)
set -o pipefail
O=gpurun_out/r5ql; mkdir -p $O
for r in 1 2; do for v in ql noql; do
  if [ $v = noql ]; then export MX_Q8_GU_NOQL=1; else unset MX_Q8_GU_NOQL; fi
  timeout -k 10 300 python -u tools/quant_step.py q4_0 q8_0 > $O/q$v$r.log 2>&1 || { tail -20 $O/q$v$r.log; exit 1; }
  grep wtype $O/q$v$r.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v run $r', d['wtype'], 'batch1', d['batch1']['ms_per_token'], 'M32', d['decode']['ms_per_step'])"
done; done
unset MX_Q8_GU_NOQL
for q in q4_0 q8_0; do
  timeout -k 10 200 python -u tools/step_probe.py --quant $q --M 1 --kinds 0,1,2,3 > $O/s$q.log 2>&1 || { tail -20 $O/s$q.log; exit 1; }
  MX_PROF_PREQUANT=1 timeout -k 10 200 python -u tools/step_probe.py --quant $q --M 1 --kinds 0,1,2,3 > $O/s${q}_pre.log 2>&1 || { tail -20 $O/s${q}_pre.log; exit 1; }
  echo "$q on-load: $(grep -o '"qkv".*' $O/s$q.log)"; echo "$q pre-quantised: $(grep -o '"qkv".*' $O/s${q}_pre.log)"
done
MX_Q8_GU_NOQL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_q8_gpu.py tests/test_q4_0_gpu.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
echo "parity with MX_Q8_GU_NOQL: $(tail -1 $O/p.log)"
