#!/bin/bash
# decode1 steady-state phase traces (graph replay) and batch-1 timing vs per-op.  tools/gpu/d1_tr.sh <tag>
OUT=gpurun_out/$1; mkdir -p $OUT
M=${MODELS:-llama3-8b,tinyllama-1.1b}
for m in ${M//,/ }; do
  for nl in ${NLS:-1}; do
    MX_D1_LOADERS=$nl timeout -k 10 200 python -u tools/d1_trace.py --model $m > $OUT/tr_${m}_l$nl.log 2>&1 || { tail -20 $OUT/tr_${m}_l$nl.log; exit 1; }
  done
done
MX_D1_LOADERS=${NL_CHECK:-1} timeout -k 10 300 python -u tools/d1_check.py --models ${D1_MODELS:-test-gqa8,test-h4096,test-tiny-ffn,$M} --steps 32 > $OUT/d1.log 2>&1 || { tail -20 $OUT/d1.log; exit 1; }
cat $OUT/d1.log
