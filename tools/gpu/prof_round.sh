# kernel-trace stats + HBM PMC passes of the default bench workload (eager launches: MX_NO_GRAPHS=1)
export TMPDIR=/tmp
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o bench -- \
  python3 bench.py --steps 16 --warmup 2 --batch1-steps 8 --prefill-prompts 0 --q8-steps 0 --no-cpu-baseline > $OUT/prof.log 2>&1 \
  || { tail -20 $OUT/prof.log; exit 1; }
tail -c 300 $OUT/prof.log
for grp in FETCH_SIZE WRITE_SIZE; do
  MX_NO_GRAPHS=1 timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pmc_$grp -o pmc -- \
    python3 bench.py --steps 4 --warmup 1 --batch1-steps 0 --prefill-prompts 0 --q8-steps 0 --no-cpu-baseline > $OUT/pmc_$grp.log 2>&1 \
    || { tail -20 $OUT/pmc_$grp.log; exit 1; }
done
echo prof_round done
