#!/bin/bash
# GPU suite, the driver's bench line, kernel stats + HBM PMC of the bench, serve_config3 via the node.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2l; mkdir -p $OUT
bash tools/gpu_round.sh r2l tests bench prof pmc || exit 1
python3 tools/prof_db.py $OUT/prof/bench_results.db --top 40 > $OUT/prof_stats.txt 2>&1 || true
timeout -k 10 300 python3 -u tools/serve_config3.py --greedy > $OUT/serve_greedy.json 2> $OUT/serve_greedy.err || { tail -20 $OUT/serve_greedy.err; exit 1; }
cat $OUT/serve_greedy.json
