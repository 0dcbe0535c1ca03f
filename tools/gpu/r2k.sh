#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2k; mkdir -p $OUT
bash tools/gpu/env_sweep.sh r2k attn_decode - "MX_ATTN_WAVES=16" "MX_ATTN_WAVES=4" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
