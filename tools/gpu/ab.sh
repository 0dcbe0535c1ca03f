timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
for c in 0 1 2 3; do MX_XS_CFG=$c timeout -k 10 120 python tools/kernel_probe.py --rows 1 > gpurun_out/probe$c.txt 2>&1; echo cfg $c; grep -E "qkv|attention" gpurun_out/probe$c.txt; done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 32 > gpurun_out/b.log 2>&1; grep -o "batch1.*" gpurun_out/b.log
