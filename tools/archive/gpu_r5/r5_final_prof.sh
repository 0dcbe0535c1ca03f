#!/bin/bash
# Final-build profiles for the driver line: kernel trace + stats of the 32-row decode (graphs off, same kernels),
# then the HBM bytes of the dominant kernel from two separate PMC passes (FETCH_SIZE, WRITE_SIZE) -> traffic.json.
#   tools/gpu/r5_final_prof.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r5prof}; mkdir -p $O
export TMPDIR=/tmp
B="bench.py --steps 16 --warmup 2 --batch1-steps 0 --tiny-tokens 0 --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --no-cpu-baseline --serve-requests 0 --geometry-steps 0"
MX_NO_GRAPHS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -- python3 $B > $O/trace.log 2>&1 || { tail -30 $O/trace.log; exit 1; }
db=$(find $O/trace -name '*.db' | head -1)
python3 tools/prof_db.py "$db" --grid --top 40 > $O/by_grid.txt && head -25 $O/by_grid.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o p -- python3 $B > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o p -- python3 $B > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
cp profiles/traffic.json $O/traffic.json
python3 tools/prof_summary.py traffic $O/fetch $O/write "void mx::mm_wide_kernel<7, 1, 2, 3>(mx::MMArgs)" $O/traffic.json llama3-8b/gate_up/M32
python3 tools/prof_summary.py pmc $O/fetch $O/write > $O/pmc_hbm.txt; head -30 $O/pmc_hbm.txt
