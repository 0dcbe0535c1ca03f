#!/bin/bash
# Config 5 on one GPU: the 70B as 8 in-process stages from a skewed split, Poisson stream; the planner
# re-splits on measured (one-stage-at-a-time) stage times
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 900 python -u tools/serve_poisson.py --model llama3-70b --stages 8 --rate 2 --n 96 --time-scale 1.0 \
  --stage-time-every 2 --parts 0:24,24:32,32:40,40:48,48:56,56:64,64:72,72:80 > $OUT/poisson70b_skew.jsonl 2> $OUT/poisson70b_skew.err \
  || { tail -n 30 $OUT/poisson70b_skew.err; exit 1; }
cat $OUT/poisson70b_skew.jsonl
