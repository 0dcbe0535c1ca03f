#!/bin/bash
# K-quant / Q4_0 parity, then the quantised decode sections and an eager kernel trace of them
#   tools/gpu/r3_kq.sh <tag>
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kquants_gpu.py tests/test_q4_0_gpu.py tests/test_q8_gpu.py -x -q \
  --timeout 240 --timeout-method thread > $OUT/kq_tests.log 2>&1 || { tail -30 $OUT/kq_tests.log; exit 1; }
tail -3 $OUT/kq_tests.log
Q="--steps 8 --warmup 2 --no-cpu-baseline --prefill-prompts 0 --tiny-tokens 0 --big-steps 0 --serve-requests 0 \
  --geometry-steps 0 --batch1-steps 0 --q8-steps 32 --kq-steps 32 --q40-steps 32"
timeout -k 10 300 python3 -u bench.py $Q > $OUT/bench_q.json 2> $OUT/bench_q.err || { tail -20 $OUT/bench_q.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_q.json'))
for k in ('q8_0','q4_k_m','q4_0'):
    if k in d: print(k, json.dumps({s: d[k][s] for s in d[k] if s in ('decode_M32','batch1','gate_up_M1','gate_up_M32')}))"
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kq -- python3 bench.py $Q --q8-steps 0 --q40-steps 0 \
  --kq-steps 8 > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 60 > $OUT/by_grid.txt && head -40 $OUT/by_grid.txt
