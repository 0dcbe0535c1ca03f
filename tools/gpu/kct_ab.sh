# wide gate/up: activation chunk of 4 vs 8 K-tiles (ring 8 vs 16 tiles per wave), 32-row decode
for i in 1 2; do
  for k in 4 8; do
    echo "kct $k: $(MX_WIDE_KCT=$k timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 32 2>&1 | tail -1)"
  done
done
