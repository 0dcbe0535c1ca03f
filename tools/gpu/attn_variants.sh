#!/bin/bash
# attention geometry variants (tools/attn_probe.py), one process each
set -o pipefail
OUT=gpurun_out/${1:-attn}
mkdir -p $OUT
MX_ATTN_V1=1 timeout -k 10 60 python -u tools/attn_probe.py > $OUT/v1.log 2>&1 || { tail $OUT/v1.log; exit 1; }
for v in 1 2 3; do
  MX_ATTN_VARIANT=$v timeout -k 10 60 python -u tools/attn_probe.py > $OUT/v$v.log 2>&1 || { tail $OUT/v$v.log; exit 1; }
done
cat $OUT/v*.log | grep variant
