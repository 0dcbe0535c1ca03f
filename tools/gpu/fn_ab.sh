# ffn RMS_NORM fused into attn_output's last work-group (opt-in MX_FUSED_NORM=1) vs its own launch, batch 1
for i in 1 2; do
  echo "fused: $(MX_FUSED_NORM=1 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1 2>&1 | tail -1)"
  echo "split: $(timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1 2>&1 | tail -1)"
done
