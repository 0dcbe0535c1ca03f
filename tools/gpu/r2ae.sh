#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2ae; mkdir -p $OUT
A="--steps 8 --warmup 2 --no-cpu-baseline --q8-steps 0 --tiny-tokens 0 --big-steps 0 --batch1-steps 0 --prefill-prompts 0"
timeout -k 10 300 python3 bench.py $A > $OUT/b.json 2> $OUT/b.err || { echo bench failed; tail $OUT/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b.json'));print(json.dumps(d['q4_k_m']))"
timeout -k 10 300 python -u -m pytest tests/test_kquants_gpu.py -x -q --timeout 300 --timeout-method thread -k "wide_rows or full_size" > $OUT/kq.log 2>&1 || { echo "kq tests failed"; tail -20 $OUT/kq.log; exit 1; }
tail -2 $OUT/kq.log
