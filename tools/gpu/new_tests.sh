#!/bin/bash
# new-test pass: the named tests (no -x), then the whole -m gpu suite with -x
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest "$@" -v -s --timeout 240 --timeout-method thread > $OUT/new.log 2>&1
rc=$?
tail -25 $OUT/new.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc2=$?
tail -15 $OUT/pytest_gpu.log
exit $(( rc > rc2 ? rc : rc2 ))
