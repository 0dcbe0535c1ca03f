#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2s; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_llama_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/llama.log 2>&1; echo "llama rc=$?"; grep -E "PASSED|FAILED|Error" $OUT/llama.log | head -20
MX_NO_FUSED_ATTN=1 timeout -k 10 300 python -u -m pytest tests/test_llama_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/llama_nf.log 2>&1; echo "llama nofused rc=$?"; grep -E "PASSED|FAILED" $OUT/llama_nf.log | head -20
