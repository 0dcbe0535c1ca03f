#!/bin/bash
# Interleaved A/B of engine builds ab/<v>.so on bench sections (3 rounds):
#   tools/gpu/ab_so.sh <tag> "<v1 v2 ...>" "<bench args>" "<python expr over d (the JSON line)>"
set -o pipefail
OUT=gpurun_out/$1; VS=$2; ARGS=$3; EXPR=$4
mkdir -p $OUT
for i in 1 2 3; do
  for v in $VS; do
    MX_LIB=$PWD/ab/$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline $ARGS > $OUT/$v.$i.json 2> $OUT/$v.$i.err \
      || { tail -20 $OUT/$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$i.json')); print('$v', $EXPR)"
  done
done
