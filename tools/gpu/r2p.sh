#!/bin/bash
# K-quant: tests, decode bench section, kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2p; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kquants_gpu.py -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest_kq.log 2>&1 || { echo "kq tests failed"; tail -60 $OUT/pytest_kq.log; exit 1; }
grep -E "prefill max|row [0-9]+:|passed|failed" $OUT/pytest_kq.log
ARGS="--steps 4 --warmup 1 --batch1-steps 4 --tiny-tokens 0 --prefill-prompts 0 --q8-steps 0 --kq-steps 32 --big-steps 0 --no-cpu-baseline"
timeout -k 10 200 python3 bench.py $ARGS > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b.json')); print(json.dumps(d['q4_k_m']))"
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kq -o kq -- python3 bench.py $ARGS > $OUT/kq.log 2>&1 || { tail -20 $OUT/kq.log; exit 1; }
python3 tools/prof_db.py $OUT/kq/kq_results.db --grid --top 40 | grep -E "mkq|q8k|attn_decode|embed" | grep -v "x128x1"
