#!/bin/bash
# Prefill MFMA counters: kernel trace + separate PMC passes over tools/prefill_probe.py (8B, 32 x 128).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2m; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/kt -o kt -- python3 tools/prefill_probe.py > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
python3 tools/prof_db.py $OUT/kt/kt_results.db --grid --top 20
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc1 -o pmc -- python3 tools/prefill_probe.py > $OUT/pmc1.log 2>&1 || { tail -20 $OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 -d $OUT/pmc2 -o pmc -- python3 tools/prefill_probe.py > $OUT/pmc2.log 2>&1 || { tail -20 $OUT/pmc2.log; exit 1; }
echo r2m done
