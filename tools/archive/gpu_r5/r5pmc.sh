set -o pipefail
O=gpurun_out/r5pmc; mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
for q in q4_0 q8_0 q4_k_m none; do
  qa=$([ $q = none ] && echo "" || echo "--quant $q")
  MX_NO_GRAPHS=1 timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/$q -o p -- python3 tools/step_probe.py $qa --kinds 2 --iters 2 > $O/$q.log 2>&1 || { tail -20 $O/$q.log; exit 1; }
  python3 tools/pmc_summary.py $O/$q --match mq8_wide mkq_wide "mm_wide_kernel<7" > $O/$q.txt; cat $O/$q.txt
done
