#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2z; mkdir -p $OUT
A="--steps 4 --warmup 2 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --big-steps 0 --batch1-steps 0"
timeout -k 10 300 python3 bench.py $A > $OUT/b.json 2> $OUT/b.err; echo "rc=$?"; grep -v "^    @" $OUT/b.err | tail -12
