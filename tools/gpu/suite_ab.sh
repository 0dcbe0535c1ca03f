#!/bin/bash
# the whole -m gpu suite on the in-tree build, then an interleaved A/B of ab/old.so vs ab/new.so
#   tools/gpu/suite_ab.sh <tag> "<bench args>" "<expr>"
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
tools/gpu/ab_so.sh $1 "old new" "$2" "$3"
