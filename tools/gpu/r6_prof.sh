#!/bin/bash
# Round 6: kernel statistics (eager launches, MX_NO_GRAPHS=1) of the 8B 32-row step, batch 1, TinyLlama and the
# Llama-2-7B geometry, then the HBM-byte PMC passes (FETCH_SIZE, WRITE_SIZE) of the 32-row step.
#   tools/gpu/r6_prof.sh <tag>
set -o pipefail
TAG=${1:-r6p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
MX_NO_GRAPHS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- \
  python3 bench.py --steps 16 --warmup 2 --batch1-steps 8 --tiny-tokens 16 --prefill-prompts 32 --q8-steps 0 --kq-steps 0 \
  --q40-steps 0 --big-steps 0 --geometry-steps 8 --serve-requests 0 --no-cpu-baseline > $OUT/prof.log 2>&1 \
  || { tail -30 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log | cut -c1-300
for grp in FETCH_SIZE WRITE_SIZE; do
  MX_NO_GRAPHS=1 timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pmc_$grp -o pmc -- \
    python3 bench.py --steps 4 --warmup 1 --batch1-steps 0 --tiny-tokens 0 --prefill-prompts 0 --q8-steps 0 --kq-steps 0 \
    --q40-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline > $OUT/pmc_$grp.log 2>&1 \
    || { tail -30 $OUT/pmc_$grp.log; exit 1; }
done
echo "r6_prof $TAG done"
