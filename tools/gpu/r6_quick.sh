#!/bin/bash
# Round 6: quick check -- the batch-invariance + sharing tests, then the bench line.
#   tools/gpu/r6_quick.sh <tag> [bench args]
set -o pipefail
TAG=${1:-r6q}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_batch_invariance_gpu.py tests/test_gpu_sharing_gpu.py -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_inv.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_inv.log; exit 1; }
tail -1 $OUT/pytest_inv.log
timeout -k 10 500 python -u bench.py "$@" > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
