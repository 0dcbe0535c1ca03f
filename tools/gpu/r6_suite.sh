#!/bin/bash
# Round 6: GPU parity suite (+ per-test durations), smoke and the bench line, one call.
#   tools/gpu/r6_suite.sh <tag> [extra pytest args]
set -o pipefail
TAG=${1:-r6}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date +%s > $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=40 "$@" \
  > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo "r6_suite $TAG done"
