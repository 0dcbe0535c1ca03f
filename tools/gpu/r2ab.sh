#!/bin/bash
# K-quant persistent GEMV: parity, then the Q4_K_M bench section with and without it
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2ab; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_kquants_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/kq.log 2>&1 || { echo "kq tests failed"; grep -E "PASSED|FAILED|Error|assert" $OUT/kq.log | tail -30; exit 1; }
grep -E "PASSED|FAILED" $OUT/kq.log
A="--steps 8 --warmup 2 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --tiny-tokens 0 --big-steps 0 --batch1-steps 0"
for v in 0 1; do
if [ $v = 1 ]; then export MX_NO_KQ_PERS=1; fi
timeout -k 10 300 python3 bench.py $A > $OUT/b$v.json 2> $OUT/b$v.err || { echo bench failed; tail $OUT/b$v.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b$v.json'));print('nopers=$v', json.dumps(d['q4_k_m']))"
done
