set -o pipefail
# engine HIP runtime initialised after PyTorch's (engine.lib): the baseline tests then a torch-using test in one process
O=gpurun_out/r5dbg; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_baseline_gpu.py tests/test_gpu_sharing_gpu.py tests/test_config5_gpu.py > $O/b.log 2>&1; echo "b rc=$?"; tail -2 $O/b.log
for o in engine-first torch-first; do timeout -k 10 120 python -u tools/hip_runtime_order_probe.py $o 2>/dev/null; done
