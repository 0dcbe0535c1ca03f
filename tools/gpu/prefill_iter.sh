#!/bin/bash
# Prefill iteration: the GEMM-path parity tests, then the bench's prefill sections and a kernel trace
#   tools/gpu/prefill_iter.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_baseline_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/pytest_prefill.log 2>&1 || { tail -30 $OUT/pytest_prefill.log; exit 1; }
tail -2 $OUT/pytest_prefill.log
ARGS="--steps 8 --warmup 2 --batch1-steps 4 --tiny-tokens 16 --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps([d.get("prefill"), d.get("tinyllama", {}).get("prefill")]))'
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o pf -- python3 bench.py $ARGS \
  > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 60 > $OUT/by_grid.txt && grep -E "gemm|attn_prefill" $OUT/by_grid.txt | head -20
