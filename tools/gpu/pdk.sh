# persistent decode kernel: parity test first (short limit), then the batch-1 bench
set -o pipefail
timeout -k 10 120 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 100 --timeout-method thread -k "persistent or decode_steps" > gpurun_out/pdk_test.log 2>&1
rc=$?
tail -25 gpurun_out/pdk_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 bench.py --seqs 1 --steps 128 --warmup 8 --batch1-steps 0 --no-cpu-baseline > gpurun_out/pdk_b1.log 2>&1 || { tail -20 gpurun_out/pdk_b1.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/pdk_b1.log
