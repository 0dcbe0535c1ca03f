# Q8_0 GEMV geometry probe (MX_Q8_CFG, kernels.hip launch_mq8_epi) at batch 1 and 32 rows
for c in 0 1 2 3 4 5 6; do
  MX_Q8_CFG=$c timeout -k 10 120 python3 tools/kernel_probe.py --q8 --rows 1 > gpurun_out/q8cfg$c.txt 2>&1 || { cat gpurun_out/q8cfg$c.txt; exit 1; }
  echo "cfg $c: $(grep -E 'qkv|attn_output|gate_up|down|lm_head' gpurun_out/q8cfg$c.txt | awk '{print $2, $3}' | tr '\n' ' ')"
done
timeout -k 10 120 python3 tools/kernel_probe.py --q8 --rows 32 > gpurun_out/q8m32.txt 2>&1 && cat gpurun_out/q8m32.txt
