# graph-mode batch-1 decode A/B: RMS_NORM-on-load vs norm kernel, interleaved runs
set -e
for i in 1 2; do
  for v in nol base; do
    if [ $v = base ]; then export MX_NO_NORM_ON_LOAD=1; else unset MX_NO_NORM_ON_LOAD; fi
    timeout -k 10 120 python3 bench.py --seqs 1 --steps 128 --warmup 8 --batch1-steps 0 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log)"
  done
done
