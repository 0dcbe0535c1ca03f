set -o pipefail
# Infinity-Cache warm (every launch on layer 0) vs cold (walk all 32 layers) per-kernel times
O=gpurun_out/r5warm; mkdir -p $O
for M in 32 1; do
timeout -k 10 200 python -u tools/step_probe.py --M $M --kinds 0,1,2,3 > $O/cold_$M.json || exit 1
MX_PROF_WARM=1 timeout -k 10 200 python -u tools/step_probe.py --M $M --kinds 0,1,2,3 > $O/warm_$M.json || exit 1
done
cat $O/*.json
