#!/bin/bash
# TinyLlama batch-1 ring-depth A/B (bench tinyllama section)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2ah; mkdir -p $OUT
A="--steps 2 --warmup 1 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --big-steps 0 --batch1-steps 0 --tiny-tokens 128"
run() {
  env $1 timeout -k 10 120 python3 bench.py $A > $OUT/t.json 2> $OUT/t.err || { echo "bench failed ($1)"; tail -5 $OUT/t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/t.json'));print('$1', d['tinyllama']['batch1']['ms_per_token'])"
}
for r in 1 2; do
run "MX_RESID_U=4"
run "MX_RESID_U=11"
run "MX_QKVXS_U=8"
run "MX_GU2048_U=8"
run "MX_GU2048_U=12"
run "MX_RESID_U=11 MX_QKVXS_U=8 MX_GU2048_U=8"
done
