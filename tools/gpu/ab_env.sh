#!/bin/bash
# A/B of one environment switch on a short bench: tools/gpu/ab_env.sh <tag> "<ENV=1 ...>" [bench args]
# Runs base / switched / base / switched, then a kernel-trace of each (eager launches).
set -o pipefail
TAG=$1; ENVB=$2; shift 2
ARGS=${@:---steps 32 --warmup 4 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --tiny-tokens 64 --big-steps 0}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python -u bench.py $ARGS > $OUT/base_$i.json 2> $OUT/base_$i.err || { tail -20 $OUT/base_$i.err; exit 1; }
  env $ENVB timeout -k 10 120 python -u bench.py $ARGS > $OUT/alt_$i.json 2> $OUT/alt_$i.err || { tail -20 $OUT/alt_$i.err; exit 1; }
  python3 -c "
import json,sys
for n in ('base','alt'):
    d=json.load(open('$OUT/%s_$i.json'%n)); t=d.get('tinyllama',{}).get('batch1',{})
    print(n, d['value'], d['ms_per_step'], d.get('batch1',{}).get('ms_per_token'), t.get('ms_per_token'))"
done
MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_base -o p -- python3 bench.py $ARGS > $OUT/prof_base.log 2>&1 || { tail -20 $OUT/prof_base.log; exit 1; }
env $ENVB MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_alt -o p -- python3 bench.py $ARGS > $OUT/prof_alt.log 2>&1 || { tail -20 $OUT/prof_alt.log; exit 1; }
echo done
