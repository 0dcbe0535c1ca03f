#!/bin/bash
# Batch-1 iteration: the bench's decode + batch-1 + TinyLlama sections, then a kernel trace of them.
#   tools/gpu/b1_iter.sh <tag> [ENV=VAL ...]  (env assignments apply to both runs)
set -o pipefail
OUT=gpurun_out/$1; shift
for kv in "$@"; do export "$kv"; done
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 16 --warmup 4 --batch1-steps 32 --tiny-tokens 128 --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({"value": d["value"], "batch1": d["batch1"], "tiny": d.get("tinyllama", {}).get("batch1")}))'
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o b1 -- python3 bench.py $ARGS \
  > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 60 > $OUT/by_grid.txt && grep -E "x1x1\]|attn_wo" $OUT/by_grid.txt | grep -v probe | head -24
