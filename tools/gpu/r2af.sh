#!/bin/bash
# persistent q|k|v GEMV at batch 1: parity (engine tests) and 8B batch-1 A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2af; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_llama_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/t.log | tail -20; exit 1; }
tail -1 $OUT/t.log
A="--steps 4 --warmup 2 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --tiny-tokens 0 --big-steps 0 --batch1-steps 64"
for r in 1 2; do for v in 0 2 3; do
MX_PERS_QKV=$v timeout -k 10 200 python3 bench.py $A > $OUT/b$v.json 2> $OUT/b$v.err || { echo bench failed; tail $OUT/b$v.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b$v.json'));print('qkv_pers=$v', d['batch1'])"
done; done
