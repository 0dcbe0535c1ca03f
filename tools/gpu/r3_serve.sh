#!/bin/bash
# Config 5 on one GPU: the Poisson driver over in-process pipeline stages, both placement
# policies (8 lanes: on one GPU the stages run one after another, so each lane streams all weights),
# one lane of 64 rows, then Llama-3-8B as a 2-stage pipeline and as one engine at the same clock.
#   tools/gpu/r3_serve.sh <tag> [n_requests] [time_scale]
set -o pipefail
OUT=gpurun_out/$1; N=${2:-64}; TS=${3:-0.25}
mkdir -p $OUT
for pol in score_aware reference; do
  timeout -k 10 500 python3 -u tools/serve_poisson.py --model llama3-70b --stages 8 --rate 2 --n $N \
    --time-scale $TS --policy $pol > $OUT/poisson70b_$pol.json 2> $OUT/poisson70b_$pol.err \
    || { tail -30 $OUT/poisson70b_$pol.err; exit 1; }
  cat $OUT/poisson70b_$pol.json
done
timeout -k 10 400 python3 -u tools/serve_poisson.py --model llama3-70b --stages 8 --lanes 1 --rows 64 --rate 2 --n $N \
  --time-scale $TS > $OUT/poisson70b_1lane.json 2> $OUT/poisson70b_1lane.err || { tail -30 $OUT/poisson70b_1lane.err; exit 1; }
cat $OUT/poisson70b_1lane.json
timeout -k 10 300 python3 -u tools/serve_poisson.py --model llama3-8b --stages 2 --rate 2 --n $N \
  --time-scale $TS > $OUT/poisson8b_2stage.json 2> $OUT/poisson8b_2stage.err \
  || { tail -30 $OUT/poisson8b_2stage.err; exit 1; }
cat $OUT/poisson8b_2stage.json
timeout -k 10 300 python3 -u tools/serve_poisson.py --model llama3-8b --replicas --rate 2 --n $N \
  --time-scale $TS > $OUT/poisson8b_replica.json 2> $OUT/poisson8b_replica.err \
  || { tail -30 $OUT/poisson8b_replica.err; exit 1; }
cat $OUT/poisson8b_replica.json
