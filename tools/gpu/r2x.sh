#!/bin/bash
# gemm3 (deeper DMA ring) vs gemm2: parity, then 4096-row and small prefills
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2x; mkdir -p $OUT
for v in 4 5; do
MX_GEMM3=$v timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_prefill" > $OUT/gemm$v.log 2>&1 || { echo "gemm$v tests failed"; tail -30 $OUT/gemm$v.log; exit 1; }
echo "v$v passed: $(grep -c PASSED $OUT/gemm$v.log)"
done
for r in 1 2; do for v in 0 4 5; do
MX_GEMM3=$v timeout -k 10 120 python3 tools/prefill_probe.py > $OUT/p$v.log 2>&1 || { echo "probe $v failed"; tail $OUT/p$v.log; exit 1; }
echo "v$v: $(tail -1 $OUT/p$v.log)"
done; done
for v in 0 4 5; do
MX_GEMM3=$v timeout -k 10 200 python3 tools/prefill_probe.py --sweep 160,256,512,1024,2048 > $OUT/s$v.log 2>&1 || { echo "sweep $v failed"; tail $OUT/s$v.log; exit 1; }
echo "v$v"; cat $OUT/s$v.log
done
