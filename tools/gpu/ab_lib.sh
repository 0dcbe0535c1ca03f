# interleaved A/B of two engine builds (ab/old.so vs ab/new.so) on the default bench workload
set -e
for i in 1 2 3; do
  for v in old new; do
    MX_LIB=$PWD/ab/$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch1-steps ${B1:-0} --prefill-prompts 0 --steps 64 > gpurun_out/ab_$v.log 2>&1
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log) $(grep -o '"batch1": {"tok_s": [0-9.]*' gpurun_out/ab_$v.log)"
  done
done
