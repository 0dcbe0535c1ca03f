# prefill GEMM v2 (LDS-DMA staging) vs v1 (register staging): parity tests, then prefill throughput
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill or gemm or 70b" > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
for v in 2 1 2 1; do
  if [ $v = 1 ]; then export MX_GEMM_V1=1; else unset MX_GEMM_V1; fi
  echo "v$v: $(timeout -k 10 200 python3 tools/prefill_probe.py 2>&1 | tail -1)"
done
