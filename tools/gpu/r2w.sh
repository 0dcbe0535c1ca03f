#!/bin/bash
# upper bound of removing the two per-layer resid_norm launches on the wide path (wrong numerics)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2w; mkdir -p $OUT
A="--steps 20 --warmup 5 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --tiny-tokens 0 --big-steps 0 --batch1-steps 0"
for i in 1 2; do
timeout -k 10 200 python3 bench.py $A > $OUT/base$i.json 2> $OUT/base$i.err || { echo base failed; tail $OUT/base$i.err; exit 1; }
MX_EXP_SKIP_NORM=1 timeout -k 10 200 python3 bench.py $A > $OUT/skip$i.json 2> $OUT/skip$i.err || { echo skip failed; tail $OUT/skip$i.err; exit 1; }
python3 -c "import json;a=json.load(open('$OUT/base$i.json'));b=json.load(open('$OUT/skip$i.json'));print('base',a['ms_per_step'],'skip',b['ms_per_step'])"
done
