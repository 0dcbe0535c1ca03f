# prefill GEMM variants (ab/*.so via MX_LIB), interleaved
for i in 1 2; do
  for v in base prio; do
    echo "$v: $(MX_LIB=$PWD/ab/$v.so timeout -k 10 200 python3 tools/prefill_probe.py 2>&1 | tail -1)"
  done
done
