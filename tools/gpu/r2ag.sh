#!/bin/bash
# TinyLlama batch-1 kernel breakdown (eager launches)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2ag; mkdir -p $OUT
cd /tmp && cd $GRAFT_REPO_ROOT
A="--steps 2 --warmup 1 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --big-steps 0 --batch1-steps 0 --tiny-tokens 16"
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run -- python3 bench.py $A > $OUT/t.json 2> $OUT/t.err || { echo failed; grep -v "^    @" $OUT/t.err | tail; exit 1; }
echo ok
