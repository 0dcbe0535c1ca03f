#!/bin/bash
# Native K-quant path: GPU tests.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2n; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kquants_gpu.py -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest_kq.log 2>&1 || { echo "kq tests failed"; tail -60 $OUT/pytest_kq.log; exit 1; }
grep -E "prefill max|row [0-9]+:|passed|failed" $OUT/pytest_kq.log
