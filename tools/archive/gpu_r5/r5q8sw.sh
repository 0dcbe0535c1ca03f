# A/B: Q8_0 17..32-row gate/up and lm_head in the swapped-operand form (MX_Q8_WSW) with the dword scale loads
# (record of a finished A/B: the switch it sets was removed from the engine afterwards -- see git log for the build it ran on)
set -o pipefail
O=gpurun_out/r5q8sw; mkdir -p $O
MX_Q8_WSW=1 MX_LIB=$PWD/ab/q8sw.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_q8_gpu.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
echo "parity (swapped Q8_0): $(tail -1 $O/p.log)"
for r in 1 2; do for v in base q8sw; do
  if [ $v = q8sw ]; then export MX_Q8_WSW=1; else unset MX_Q8_WSW; fi
  MX_LIB=$PWD/ab/$v.so timeout -k 10 200 python -u tools/step_probe.py --quant q8_0 --M 32 --kinds 2,4 > $O/s$v$r.log 2>&1 || { tail -20 $O/s$v$r.log; exit 1; }
  echo "$v run $r $(grep -o '"gate_up".*' $O/s$v$r.log)"
done; done
