#!/bin/bash
# Round-4 pipeline evidence on one GPU: the multi-process bench path with host-staged hand-offs
# (tests/test_pipeline_rehearsal_gpu.py), then config 5's Poisson stream on the 70B as 8 in-process
# stages started from a skewed split (the stage planner's re-split, p2p:156-168).
#   tools/gpu/r4_pipeline.sh <tag>
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_pipeline_rehearsal_gpu.py -x -v -s --timeout 330 --timeout-method thread \
  > $OUT/rehearsal.log 2>&1 || { tail -40 $OUT/rehearsal.log; exit 1; }
tail -5 $OUT/rehearsal.log
timeout -k 10 420 python -u tools/serve_poisson.py --model llama3-70b --stages 8 --rate 2 --n 64 --time-scale 0.25 \
  --parts 0:24,24:32,32:40,40:48,48:56,56:64,64:72,72:80 > $OUT/poisson70b_skew.jsonl 2> $OUT/poisson70b_skew.err \
  || { tail -30 $OUT/poisson70b_skew.err; exit 1; }
cat $OUT/poisson70b_skew.jsonl
