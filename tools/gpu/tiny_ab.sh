# TinyLlama-1.1B batch-1 decode: default kernels vs the persistent decode kernel (MX_PDK=1)
set -e
for i in 1 2; do
  echo "default $(timeout -k 10 120 python3 tools/q8_decode.py --model tinyllama-1.1b --bf16 --rows 1 --steps 128)"
  echo "pdk     $(MX_PDK=1 timeout -k 10 120 python3 tools/q8_decode.py --model tinyllama-1.1b --bf16 --rows 1 --steps 128)"
  echo "nopers  $(MX_NO_PERS=1 timeout -k 10 120 python3 tools/q8_decode.py --model tinyllama-1.1b --bf16 --rows 1 --steps 128)"
done
