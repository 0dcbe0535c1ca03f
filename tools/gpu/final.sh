# round-end refresh: the copy-peak probe alone, the full bench line, and (with "serve") config 3
# through the node.  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
OUT=gpurun_out/final
mkdir -p $OUT
timeout -k 10 60 python -u bench.py --copy-peak-only > $OUT/copy.log 2>&1 || { tail -30 $OUT/copy.log; exit 1; }
cat $OUT/copy.log
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [ "$1" = serve ]; then
  timeout -k 10 300 python -u tools/serve_config3.py > $OUT/serve3.log 2>&1 || { tail -30 $OUT/serve3.log; exit 1; }
  tail -1 $OUT/serve3.log
fi
