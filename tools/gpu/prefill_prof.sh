# prefill: GEMM-path parity tests, then a rocprofv3 kernel trace of tools/prefill_probe.py
export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py tests/test_q8_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill or gemm or 70b" > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
timeout -k 10 200 python3 tools/prefill_probe.py 2>&1 | tail -1
MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pf -o pf -- python3 tools/prefill_probe.py > gpurun_out/pf.log 2>&1
tail -1 gpurun_out/pf.log
