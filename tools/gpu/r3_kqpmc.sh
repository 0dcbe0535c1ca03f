#!/bin/bash
# Why the one-token quantised GEMVs sit below the HBM roofline: per-kernel timing (kernel_probe) and
# SQ issue/wait counters in passes of their own, for Q4_K_M, Q4_0, Q8_0 and bf16 gate/up / down.
#   tools/gpu/r3_kqpmc.sh <tag>
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
for w in q4_k_m q4_0 q8_0 bf16; do
  WA=""; [ $w != bf16 ] && WA="--wtype $w"
  timeout -k 10 120 python3 tools/kernel_probe.py $WA --rows 1,32 --kinds 0,1,2,3 --iters 20 > $OUT/probe_$w.txt 2>&1 \
    || { tail -20 $OUT/probe_$w.txt; exit 1; }
  cat $OUT/probe_$w.txt | grep 'M='
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VMEM"; do
    n=$(echo $P | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/pmc_${w}_$n -o pmc -- python3 tools/kernel_probe.py $WA --rows 1 \
      --kinds 2,3 --iters 5 > $OUT/pmc_${w}_$n.log 2>&1 || { tail -20 $OUT/pmc_${w}_$n.log; exit 1; }
    python3 tools/prof_summary.py pmc $OUT/pmc_${w}_$n > $OUT/pmc_${w}_$n.txt 2>&1 || exit 1
    rm -rf $OUT/pmc_${w}_$n
  done
done
