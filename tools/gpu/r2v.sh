#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2v; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_prefill" > $OUT/gemm.log 2>&1 || { echo "gemm tests failed"; tail -30 $OUT/gemm.log; exit 1; }
grep -cE "PASSED" $OUT/gemm.log
timeout -k 10 300 python -u tools/prefill_probe.py --sweep 80,128,160,256,384,512,1024 --targets 256,128,512 > $OUT/sweep.log 2>&1 || { echo "sweep failed"; tail -20 $OUT/sweep.log; exit 1; }
cat $OUT/sweep.log
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/p160 -o run -- python3 tools/prefill_probe.py --sweep 160 --targets 256 > $OUT/p160.log 2>&1 || { echo "p160 failed"; tail -20 $OUT/p160.log; exit 1; }
MX_SCHED_TRACE=1 timeout -k 10 300 python -u tools/serve_config3.py --greedy > $OUT/serve.json 2> $OUT/serve.err || { echo "serve failed"; tail -20 $OUT/serve.err; exit 1; }
cat $OUT/serve.json; grep -m 8 "sched:" $OUT/serve.err
