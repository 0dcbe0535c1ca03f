#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2i; mkdir -p $OUT
for P in 1 2; do
  MX_ATTN_PIPE=$P MX_ATTN_TRACE=1 timeout -k 10 60 python -u tools/attn_probe.py > $OUT/attn_trace$P.log 2>&1 || { tail $OUT/attn_trace$P.log; exit 1; }
  echo "PIPE=$P"; grep "attn trace" $OUT/attn_trace$P.log
done
bash tools/gpu/env_sweep.sh r2i attn - "MX_ATTN_PIPE=2" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
