#!/bin/bash
# decode1 (persistent one-token launch) vs the per-op kernels: parity + batch-1 timing with one and
# two loader waves, then the phase traces.   tools/gpu/d1_ab.sh <tag>
OUT=gpurun_out/$1; mkdir -p $OUT
M=${MODELS:-test-gqa8,test-h4096,test-tiny-ffn,llama3-8b,tinyllama-1.1b}
MX_D1_LOADERS=1 timeout -k 10 300 python -u tools/d1_check.py --models $M --steps 32 > $OUT/d1_l1.log 2>&1 || { tail -20 $OUT/d1_l1.log; exit 1; }
MX_D1_LOADERS=2 timeout -k 10 300 python -u tools/d1_check.py --models $M --steps 32 > $OUT/d1_l2.log 2>&1 || { tail -20 $OUT/d1_l2.log; exit 1; }
for m in llama3-8b tinyllama-1.1b; do
  for nl in 1 2; do
    MX_D1_LOADERS=$nl timeout -k 10 200 python -u tools/d1_trace.py --model $m > $OUT/tr_${m}_l$nl.log 2>&1 || { tail -20 $OUT/tr_${m}_l$nl.log; exit 1; }
  done
done
cat $OUT/d1_l1.log $OUT/d1_l2.log
