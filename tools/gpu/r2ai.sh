#!/bin/bash
# K-quant quantise-on-load at batch 1: parity, then Q4_K_M batch-1 A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2ai; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kquants_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/kq.log 2>&1 || { echo "kq tests failed"; grep -E "PASSED|FAILED|Error|assert" $OUT/kq.log | tail -30; exit 1; }
grep -cE "PASSED" $OUT/kq.log
A="--steps 8 --warmup 2 --no-cpu-baseline --q8-steps 0 --tiny-tokens 0 --big-steps 0 --batch1-steps 0 --prefill-prompts 0"
for r in 1 2; do for v in 0 1; do
if [ $v = 1 ]; then export MX_KQ_NO_QL=1; else unset MX_KQ_NO_QL; fi
timeout -k 10 300 python3 bench.py $A > $OUT/b$v.json 2> $OUT/b$v.err || { echo bench failed; tail $OUT/b$v.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b$v.json'));q=d['q4_k_m'];print('no_ql=$v', q['batch1'], q['decode_M32']['ms_per_step'])"
done; done
