#!/bin/bash
# Full GPU suite, bench line (with the Q4_K_M section), K-quant kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2o; mkdir -p $OUT
bash tools/gpu_round.sh r2o tests bench || exit 1
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kq -o kq -- python3 bench.py --steps 4 --warmup 1 --batch1-steps 4 --tiny-tokens 0 --prefill-prompts 0 --q8-steps 0 --kq-steps 16 --big-steps 0 --no-cpu-baseline > $OUT/kq.log 2>&1 || { tail -20 $OUT/kq.log; exit 1; }
python3 tools/prof_db.py $OUT/kq/kq_results.db --grid --top 40 > $OUT/kq_stats.txt
head -30 $OUT/kq_stats.txt
