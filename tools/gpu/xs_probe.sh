# RMS_NORM-on-load geometry probe at batch 1 (kinds: 0 qkv, 2 gate/up, 5 qkv+XS, 6 gate/up+XS)
for c in 0 1 3 4; do
  MX_XS_CFG=$c timeout -k 10 100 python3 tools/kernel_probe.py --rows 1 > gpurun_out/xs$c.txt 2>&1
  echo "cfg $c: $(grep -E 'qkv|gate_up' gpurun_out/xs$c.txt | awk '{print $2, $3}' | tr '\n' ' ')"
done
