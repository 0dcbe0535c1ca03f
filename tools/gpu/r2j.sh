#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2j; mkdir -p $OUT
MX_ATTN_TRACE=1 timeout -k 10 60 python -u tools/attn_probe.py > $OUT/attn_trace.log 2>&1 || { tail $OUT/attn_trace.log; exit 1; }
grep "attn trace" $OUT/attn_trace.log
bash tools/gpu/env_sweep.sh r2j attn - || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
