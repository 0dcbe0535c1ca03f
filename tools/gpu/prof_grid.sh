#!/bin/bash
# Kernel trace of the bench's decode sections (eager launches, MX_NO_GRAPHS=1) with per-grid stats:
#   tools/gpu/prof_grid.sh <tag> [bench args...]
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
MX_NO_GRAPHS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- \
  python3 bench.py --steps 16 --warmup 2 --batch1-steps 8 --tiny-tokens 16 --prefill-prompts 0 --q8-steps 0 \
  --kq-steps 0 --q40-steps 0 --big-steps 0 --no-cpu-baseline --serve-requests 0 --geometry-steps 0 "$@" > $OUT/prof.log 2>&1 \
  || { tail -30 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 80 > $OUT/by_grid.txt && head -45 $OUT/by_grid.txt
