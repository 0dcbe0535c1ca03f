set -o pipefail
O=gpurun_out/r5c5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_config5_gpu.py tests/test_pipeserve_resplit_gpu.py -x -v -s --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED|lanes_used|history" $O/pytest.log
bash tools/gpu/r5_poisson.sh r5c5
