# decode attention waves per (kv head, row): 8 (default) vs 4, at 32 rows and batch 1 (graph replay)
for i in 1 2; do
  for nw in 8 4; do
    echo "nw $nw: $(MX_ATTN_WAVES=$nw timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 32 2>&1 | tail -1) | $(MX_ATTN_WAVES=$nw timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1 2>&1 | tail -1)"
  done
done
