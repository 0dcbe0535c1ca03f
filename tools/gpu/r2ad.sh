#!/bin/bash
# K-quant prefill through dequantised bf16 GEMMs: parity + the Q4_K_M bench section
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2ad; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kquants_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/kq.log 2>&1 || { echo "kq tests failed"; grep -E "PASSED|FAILED|Error|assert" $OUT/kq.log | tail -30; exit 1; }
grep -E "PASSED|FAILED" $OUT/kq.log | tail -8
A="--steps 8 --warmup 2 --no-cpu-baseline --q8-steps 0 --tiny-tokens 0 --big-steps 0 --batch1-steps 0"
timeout -k 10 300 python3 bench.py $A > $OUT/b.json 2> $OUT/b.err || { echo bench failed; tail $OUT/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b.json'));print(json.dumps(d['q4_k_m']));print(json.dumps(d['prefill']))"
