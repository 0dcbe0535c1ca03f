#!/bin/bash
# split-K prefill GEMM: parity, small-prompt sweep, config-3 serving through the handler
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2t; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_prefill" > $OUT/gemm.log 2>&1 || { echo "gemm tests failed"; tail -30 $OUT/gemm.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/gemm.log
timeout -k 10 300 python -u tools/prefill_probe.py --sweep 64,80,128,160,256,384,512,1024,2048 --targets 256,0,128,512 > $OUT/sweep.log 2>&1 || { echo "sweep failed"; tail -20 $OUT/sweep.log; exit 1; }
cat $OUT/sweep.log
MX_SCHED_TRACE=1 timeout -k 10 300 python -u tools/serve_config3.py --greedy > $OUT/serve.json 2> $OUT/serve.err || { echo "serve failed"; tail -20 $OUT/serve.err; exit 1; }
cat $OUT/serve.json; grep -m 12 "sched:" $OUT/serve.err
