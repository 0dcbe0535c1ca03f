#!/bin/bash
# decode1 variant build (ab/<v>.so) vs the tree's build: batch-1 steady-state traces and timing.
#   tools/gpu/d1_var.sh <tag> <v> [env assignments for the variant]
OUT=gpurun_out/$1; V=$2; shift 2; mkdir -p $OUT
for m in llama3-8b tinyllama-1.1b; do
  env MX_LIB=$PWD/ab/$V.so "$@" timeout -k 10 200 python -u tools/d1_trace.py --model $m > $OUT/tr_${m}_$V.log 2>&1 || { tail -20 $OUT/tr_${m}_$V.log; exit 1; }
  timeout -k 10 200 python -u tools/d1_trace.py --model $m > $OUT/tr_${m}_base.log 2>&1 || { tail -20 $OUT/tr_${m}_base.log; exit 1; }
done
env MX_LIB=$PWD/ab/$V.so "$@" timeout -k 10 300 python -u tools/d1_check.py --models test-gqa8,test-h4096,llama3-8b,tinyllama-1.1b --steps 32 > $OUT/d1_$V.log 2>&1 || { tail -20 $OUT/d1_$V.log; exit 1; }
cat $OUT/d1_$V.log
