#!/bin/bash
# Q4_K_M batch-1 / 32-row kernel breakdown (bench q4_k_m section, eager launches)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2ac; mkdir -p $OUT
cd /tmp && cd $GRAFT_REPO_ROOT
A="--steps 4 --warmup 1 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --tiny-tokens 0 --big-steps 0 --batch1-steps 0 --kq-steps 8"
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kq -o run -- python3 bench.py $A > $OUT/kq.json 2> $OUT/kq.err || { echo failed; grep -v "^    @" $OUT/kq.err | tail; exit 1; }
echo ok
