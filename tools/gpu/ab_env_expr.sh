#!/bin/bash
# Interleaved A/B of engine environment settings (3 rounds), printing a python expression over the line d:
#   tools/gpu/ab_env_expr.sh <tag> "<ENV=a ENV=b ...>" "<bench args>" "<expr>"
# each word of the 2nd argument is one variant: a comma-separated list of VAR=value (or "-" for none)
set -o pipefail
OUT=gpurun_out/$1; VS=$2; ARGS=$3; EXPR=$4
mkdir -p $OUT
for i in 1 2 3; do
  for v in $VS; do
    envs=$( [ "$v" = "-" ] && echo "" || echo "$v" | tr ',' ' ')
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline $ARGS > $OUT/$v.$i.json 2> $OUT/$v.$i.err \
      || { tail -20 $OUT/$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$i.json')); print('$v', $EXPR)"
  done
done
