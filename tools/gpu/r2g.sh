#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2g; mkdir -p $OUT
MX_ATTN_TRACE=1 timeout -k 10 60 python -u tools/attn_probe.py > $OUT/attn_trace.log 2>&1 || { tail $OUT/attn_trace.log; exit 1; }
grep "attn trace" $OUT/attn_trace.log
ARGS="--steps 32 --warmup 4 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --tiny-tokens 64 --big-steps 0"
for E in "MX_NOP=1" "MX_PREFETCH=1" "MX_PREFETCH=1 MX_PREFETCH_MB=8" "MX_PREFETCH=1 MX_PREFETCH_MB=64" "MX_PREFETCH=1 MX_PREFETCH_WG=64" "MX_NOP=1"; do
  env $E timeout -k 10 120 python -u bench.py $ARGS > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b.json')); t=d.get('tinyllama',{}).get('batch1',{})
print('$E', 'M32 ms', d['ms_per_step'], 'b1 ms', d.get('batch1',{}).get('ms_per_token'), 'tiny ms', t.get('ms_per_token'))"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
