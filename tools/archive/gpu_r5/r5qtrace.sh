# kernel traces of the quantised 32-sequence decode steps at the final build (tools/quant_step.py, graphs off)
set -o pipefail
O=gpurun_out/r5qtrace; mkdir -p $O; export TMPDIR=/tmp
for q in q4_0 q8_0; do
  MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$q -o p -- python3 tools/quant_step.py $q --steps 8 > $O/$q.log 2>&1 || { tail -20 $O/$q.log; exit 1; }
  python3 tools/prof_db.py "$(find $O/$q -name '*.db' | head -1)" --grid --top 30 > $O/$q.txt && head -3 $O/$q.txt
done
