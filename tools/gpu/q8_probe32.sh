# Q8_0 32-row GEMV geometry probe (MX_Q8_CFG2, kernels.hip launch_mq8_epi)
for c in 0 1 2 3 4; do
  MX_Q8_CFG2=$c timeout -k 10 120 python3 tools/kernel_probe.py --q8 --rows 32 > gpurun_out/q8c2_$c.txt 2>&1 || { cat gpurun_out/q8c2_$c.txt; exit 1; }
  echo "cfg $c: $(grep -E 'qkv|attn_output|gate_up|down|lm_head' gpurun_out/q8c2_$c.txt | awk '{print $2, $3}' | tr '\n' ' ')"
done
