set -o pipefail
O=gpurun_out/r5qg; mkdir -p $O; export TMPDIR=/tmp
for v in $VARIANTS; do
  MX_LIB=$PWD/ab/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_q8_gpu.py tests/test_q4_0_gpu.py -k "gemm" > $O/p$v.log 2>&1 || { tail -20 $O/p$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/p$v.log)"
done
for q in q8_0 q4_0; do for v in $VARIANTS; do
  MX_LIB=$PWD/ab/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t$v$q -o p -- python3 tools/prefill_probe.py --quant $q > $O/t$v$q.log 2>&1 || { tail -20 $O/t$v$q.log; exit 1; }
  db=$(find $O/t$v$q -name '*.db' | head -1)
  echo "$q $v $(grep 'tok/s' $O/t$v$q.log | tail -1)"; python3 tools/prof_db.py "$db" --match q8gemm --top 6 | tail -n +2 | cut -c1-120
done; done
