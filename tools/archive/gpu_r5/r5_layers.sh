set -o pipefail
O=gpurun_out/r5layers; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_fulldepth_stages_gpu.py -k "70b_sampled or 8b_every" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "layer|PASSED|passed|worst" $O/pytest.log | tail -45
