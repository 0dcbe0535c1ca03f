#!/bin/bash
# kernel breakdown of a 160-row (split-K) and a 4096-row prefill
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2u; mkdir -p $OUT
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p160 -o run -- python3 tools/prefill_probe.py --sweep 160 --targets 256 > $OUT/p160.log 2>&1 || { echo "p160 failed"; tail -20 $OUT/p160.log; exit 1; }
cat $OUT/p160.log | grep target
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p4096 -o run -- python3 tools/prefill_probe.py > $OUT/p4096.log 2>&1 || { echo "p4096 failed"; tail -20 $OUT/p4096.log; exit 1; }
cat $OUT/p4096.log | grep tok
find $OUT -name "*stats*" | head
