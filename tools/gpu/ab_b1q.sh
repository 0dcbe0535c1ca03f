# interleaved A/B of two engine builds (ab/old.so vs ab/new.so) and new.so with MX_NO_PERS=1:
# batch-1 bf16 decode, graph replay
set -e
for i in 1 2 3; do
  echo "base $(MX_NO_PERS=1 MX_LIB=$PWD/ab/new.so timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
  for v in old new; do
    echo "$v $(MX_LIB=$PWD/ab/$v.so timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows ${ROWS:-1})"
  done
done
