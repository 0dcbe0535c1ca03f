#!/bin/bash
# One GPU measurement pass: gpu parity tests, bench line, rocprofv3 kernel stats of the
# same bench (eager launches: MX_NO_GRAPHS=1), then HBM-byte PMC passes (one counter
# group per pass).  Every GPU step has its own time limit; the first failure ends it.
#   tools/gpu_round.sh <tag> [tests|bench|prof|pmc ...]
set -o pipefail
TAG=${1:-r1}; shift
STEPS=${@:-tests bench prof pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
      tail -3 $OUT/pytest_gpu.log ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || { tail -30 $OUT/smoke.log; exit 1; }
      tail -2 $OUT/smoke.log ;;
    bench)
      timeout -k 10 450 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
      tail -1 $OUT/bench.log ;;
    prof)
      MX_NO_GRAPHS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- \
        python3 bench.py --steps 16 --warmup 2 --batch1-steps 8 --tiny-tokens 16 --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline > $OUT/prof.log 2>&1 \
        || { tail -30 $OUT/prof.log; exit 1; }
      tail -1 $OUT/prof.log ;;
    pmc)
      for grp in FETCH_SIZE WRITE_SIZE; do
        MX_NO_GRAPHS=1 timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pmc_$grp -o pmc -- \
          python3 bench.py --steps 4 --warmup 1 --batch1-steps 0 --tiny-tokens 0 --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --no-cpu-baseline > $OUT/pmc_$grp.log 2>&1 \
          || { tail -30 $OUT/pmc_$grp.log; exit 1; }
      done ;;
  esac
done
echo "gpu_round $TAG done"
