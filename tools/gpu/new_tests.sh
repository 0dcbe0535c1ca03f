#!/bin/bash
# Run selected GPU tests (one pytest process), log under gpurun_out/<tag>/.
#   tools/gpu/new_tests.sh <tag> <pytest args...>
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
tail -40 $OUT/pytest.log
exit $rc
