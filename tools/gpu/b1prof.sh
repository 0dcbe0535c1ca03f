# batch-1 decode kernel profile, with and without RMS_NORM-on-load (eager launches for rocprofv3)
export TMPDIR=/tmp
set -e
for v in nol base; do
  if [ $v = base ]; then export MX_NO_NORM_ON_LOAD=1; fi
  MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/b1_$v -o b1 -- python3 bench.py --seqs 1 --steps 32 --warmup 2 --batch1-steps 0 --no-cpu-baseline > gpurun_out/b1_$v.log 2>&1
  grep -o '"value": [0-9.]*' gpurun_out/b1_$v.log
done
