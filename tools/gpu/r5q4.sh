set -o pipefail
O=gpurun_out/r5q4; mkdir -p $O
for r in 2 4 2 4; do
  MX_Q4_RING=$r timeout -k 10 200 python -u tools/step_probe.py --quant q4_0 --kinds 2,0,1,3 > $O/q4_ring$r.json 2>$O/err.txt || { tail $O/err.txt; exit 1; }
  echo "ring $r $(cat $O/q4_ring$r.json)"
done
timeout -k 10 200 python -u tools/step_probe.py --quant q4_k_m --kinds 2,0,1,3 > $O/q4km.json 2>$O/err.txt || exit 1
cat $O/q4km.json
timeout -k 10 200 python -u tools/step_probe.py --quant q8_0 --kinds 2,0,1,3 > $O/q8.json 2>$O/err.txt || exit 1
cat $O/q8.json
bash tools/gpu/r5attn.sh
