# split-K target A/B for the 17..32-row quantised attn_output / ffn_down / q|k|v (MX_SLAB_TARGET), whole
# decode steps (tools/quant_step.py), then a kernel trace of the Q4_K_M step at the default target
set -o pipefail
O=gpurun_out/r5slab; mkdir -p $O; export TMPDIR=/tmp
for t in 256 512 1024; do
  MX_SLAB_TARGET=$t timeout -k 10 300 python -u tools/quant_step.py q4_k_m q8_0 q4_0 > $O/t$t.log 2>&1 || { tail -20 $O/t$t.log; exit 1; }
  grep wtype $O/t$t.log | cut -c1-200
done
MX_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kq -o p -- python3 tools/quant_step.py q4_k_m --steps 8 > $O/kq.log 2>&1 || { tail -20 $O/kq.log; exit 1; }
python3 tools/prof_db.py "$(find $O/kq -name '*.db' | head -1)" --top 14 | cut -c1-150
