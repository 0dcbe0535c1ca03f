#!/bin/bash
# Q8_0 / Q4_0 iteration: their parity tests, then the bench's Q8_0 and Q4_0 sections alone and their
# per-grid kernel trace (eager launches).   tools/gpu/q8_iter.sh <tag> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/$1; K=${2:-}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_q8_gpu.py tests/test_q4_0_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_q8.log 2>&1 || { tail -30 $OUT/pytest_q8.log; exit 1; }
tail -2 $OUT/pytest_q8.log
ARGS="--steps 16 --warmup 2 --batch1-steps 4 --tiny-tokens 0 --prefill-prompts 0 --kq-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $ARGS --q8-steps 32 --q40-steps 32 > $OUT/bench_kq.log 2>&1 || { tail -30 $OUT/bench_kq.log; exit 1; }
tail -1 $OUT/bench_kq.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps([d.get("q8_0"), d.get("q4_0")]))'
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kq -- python3 bench.py $ARGS --q8-steps 8 --q40-steps 8 \
  > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 60 > $OUT/by_grid.txt && grep -E "mq8|norm_q8|quantize_q8|attn_decode_kernel<128, 4, 8, false>|embed" $OUT/by_grid.txt | head -30
