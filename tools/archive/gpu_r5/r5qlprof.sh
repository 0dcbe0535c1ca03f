# profile_kernel at one token now times the quantise-on-load GEMVs the decode runs (MX_PROF_PREQUANT=1: the old form)
set -o pipefail
O=gpurun_out/r5qlprof; mkdir -p $O
for q in q4_k_m q4_0 q8_0; do
  timeout -k 10 200 python -u tools/step_probe.py --quant $q --M 1 --kinds 0,1,2,3 > $O/s$q.log 2>&1 || { tail -20 $O/s$q.log; exit 1; }
  MX_PROF_PREQUANT=1 timeout -k 10 200 python -u tools/step_probe.py --quant $q --M 1 --kinds 0,1,2,3 > $O/s${q}_pre.log 2>&1 || { tail -20 $O/s${q}_pre.log; exit 1; }
  echo "$q on-load: $(grep -o '"qkv".*' $O/s$q.log)"; echo "$q pre-quantised: $(grep -o '"qkv".*' $O/s${q}_pre.log)"
done
