#!/bin/bash
# Q8_0 prompt GEMM iteration: the Q8_0 parity tests, then the bench's q8_0 section and a kernel trace
#   tools/gpu/q8gemm_iter.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_q8_gpu.py tests/test_q4_0_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_q8.log 2>&1 || { tail -40 $OUT/pytest_q8.log; exit 1; }
tail -2 $OUT/pytest_q8.log
ARGS="--steps 2 --warmup 1 --batch1-steps 0 --tiny-tokens 0 --q8-steps 4 --kq-steps 0 --q40-steps 4 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); [print(k, d[k]["prefill"]["tok_s"], d[k]["decode_M32"]["tok_s"], d[k]["gate_up_M32"]["us_per_launch"], d[k]["gate_up_M32"]["frac"], d[k]["batch1"]["tok_s"]) for k in ("q8_0", "q4_0")]'
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o q8 -- python3 bench.py $ARGS \
  > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 40 > $OUT/by_grid.txt && grep -E "q8gemm|mq8" $OUT/by_grid.txt | head -12
