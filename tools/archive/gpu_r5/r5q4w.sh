# A/B of 17-32-row quantised GEMV builds (ab/<variant>.so): parity of the quantised GPU tests, then
# tools/step_probe.py per-kernel times at 32 rows.  VARIANTS="base x" QUANT=q4_0 TESTS="tests/test_q4_0_gpu.py"
set -o pipefail
O=gpurun_out/r5q4w; mkdir -p $O; export TMPDIR=/tmp
for v in $VARIANTS; do
  MX_LIB=$PWD/ab/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $O/p$v.log 2>&1 || { tail -20 $O/p$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/p$v.log)"
done
for r in 1 2; do for v in $VARIANTS; do
  MX_LIB=$PWD/ab/$v.so timeout -k 10 200 python -u tools/step_probe.py --quant $QUANT --M 32 --kinds ${KINDS:-2,4} > $O/s$v$r.log 2>&1 || { tail -20 $O/s$v$r.log; exit 1; }
  echo "$v run $r: $(tr '\n' ' ' < $O/s$v$r.log | cut -c1-300)"
done; done
