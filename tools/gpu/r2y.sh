#!/bin/bash
# batch-1 kernel breakdown: 8B and TinyLlama (bench sections) under a kernel trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2y; mkdir -p $OUT
cd /tmp && cd $GRAFT_REPO_ROOT
A="--steps 4 --warmup 2 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --big-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/b8 -o run -- python3 bench.py $A --tiny-tokens 0 > $OUT/b8.json 2> $OUT/b8.err || { echo failed8; grep -v "^    @" $OUT/b8.err | tail; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/bt -o run -- python3 bench.py $A --batch1-steps 0 > $OUT/bt.json 2> $OUT/bt.err || { echo failedt; grep -v "^    @" $OUT/bt.err | tail; }
ls $OUT/b8 $OUT/bt
