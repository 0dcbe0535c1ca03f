# HBM bytes (PMC FETCH_SIZE / WRITE_SIZE, separate passes) of the quantised decode kernels at the final build:
# Q4_0 and Q8_0 32-sequence steps + batch 1 (tools/quant_step.py, graphs off)
set -o pipefail
O=gpurun_out/r5qpmc; mkdir -p $O; export TMPDIR=/tmp
for q in q4_0 q8_0; do
  MX_NO_GRAPHS=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/$q-fetch -o p -- python3 tools/quant_step.py $q --steps 4 > $O/$q-fetch.log 2>&1 || { tail -20 $O/$q-fetch.log; exit 1; }
  MX_NO_GRAPHS=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/$q-write -o p -- python3 tools/quant_step.py $q --steps 4 > $O/$q-write.log 2>&1 || { tail -20 $O/$q-write.log; exit 1; }
  python3 tools/prof_summary.py pmc $O/$q-fetch $O/$q-write > $O/$q-pmc.txt && grep -E "wsw|pers_ql|mq8_wide|mq8_kernel" $O/$q-pmc.txt | head -8
done
