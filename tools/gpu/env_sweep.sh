#!/bin/bash
# Short bench + eager kernel trace per environment setting:
#   tools/gpu/env_sweep.sh <tag> <match> "ENV_A=1" "ENV_B=2" ...   ("-" = no extra env)
# Prints the bench numbers and the kernels whose name contains <match> (tools/prof_db.py).
set -o pipefail
TAG=$1; MATCH=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 32 --warmup 4 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --tiny-tokens 64 --big-steps 0"
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E="MX_NOP=1"
  env $E timeout -k 10 120 python -u bench.py $ARGS > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b$i.json')); t=d.get('tinyllama',{}).get('batch1',{})
print('$E', 'M32 ms', d['ms_per_step'], 'b1 ms', d.get('batch1',{}).get('ms_per_token'), 'tiny ms', t.get('ms_per_token'))"
  env $E MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/p$i -o p -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
  python3 tools/prof_db.py $OUT/p$i/p_results.db --grid --match "$MATCH" --top 12
done
