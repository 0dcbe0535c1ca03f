# Q8_0 batch-1 geometry A/B: quantise-on-load sites and rows per work-group
for v in "0 1" "4 1" "0 2" "4 2" "20 1" "0 1"; do
  set -- $v
  echo "mask $1 rt $2: $(MX_Q8_NO_QL_MASK=$1 MX_Q8_QL_RT=$2 timeout -k 10 120 python3 tools/q8_decode.py --rows 1 2>&1 | tail -1)"
done
