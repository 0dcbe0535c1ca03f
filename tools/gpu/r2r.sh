#!/bin/bash
# fused one-token qkv+attention: equivalence test, full suite, A/B bench + trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2r; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -k fused --timeout 120 --timeout-method thread > $OUT/fused.log 2>&1 || { echo "fused test failed"; tail -40 $OUT/fused.log; exit 1; }
tail -2 $OUT/fused.log
bash tools/gpu/env_sweep.sh r2r attn - MX_NO_FUSED_ATTN=1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
