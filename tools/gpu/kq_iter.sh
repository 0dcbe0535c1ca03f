#!/bin/bash
# K-quant iteration: the K-quant / Q4_0 parity tests, then the bench's Q4_K_M section alone and its
# per-grid kernel trace (eager launches).   tools/gpu/kq_iter.sh <tag> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/$1; K=${2:-}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kquants_gpu.py tests/test_q4_0_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_kq.log 2>&1 || { tail -30 $OUT/pytest_kq.log; exit 1; }
tail -2 $OUT/pytest_kq.log
ARGS="--steps 16 --warmup 2 --batch1-steps 4 --tiny-tokens 0 --prefill-prompts 0 --q8-steps 0 --q40-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $ARGS --kq-steps 32 > $OUT/bench_kq.log 2>&1 || { tail -30 $OUT/bench_kq.log; exit 1; }
tail -1 $OUT/bench_kq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('q4_k_m')))"
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kq -- python3 bench.py $ARGS --kq-steps 8 \
  > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 60 > $OUT/by_grid.txt && grep -E "mkq|q8k|attn_decode_kernel<128, 4, 8, false>|embed" $OUT/by_grid.txt | head -30
