#!/bin/bash
# Q4_K_M decode A/B: bench section + eager kernel trace per environment setting.
#   tools/gpu/kq_sweep.sh <tag> "ENV_A=1" "ENV_B=2" ...   ("-" = no extra env)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --batch1-steps 2 --no-cpu-baseline --prefill-prompts 0 --q8-steps 0 --kq-steps 32 --tiny-tokens 0 --big-steps 0"
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E="MX_NOP=1"
  env $E timeout -k 10 150 python -u bench.py $ARGS > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b$i.json'))['q4_k_m']
print('$E', 'M32 ms', d['decode_M32']['ms_per_step'], 'b1 ms', d['batch1']['ms_per_token'], 'gu1 us', d['gate_up_M1']['us_per_launch'], 'gu32 us', d['gate_up_M32']['us_per_launch'])"
  env $E MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/p$i -o p -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
  python3 tools/prof_db.py $OUT/p$i/p_results.db --grid --top 30 | grep -E "mkq|q8k|attn_decode|embed" | grep -v "x128x1\|x4096x1"
done
