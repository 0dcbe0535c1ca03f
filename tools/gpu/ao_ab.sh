# fused attention+attn_output (opt-in MX_ATTN_O=1) at batch 1 (graph replay): poll interval /
# prefetch variants vs the two-launch default
run() { timeout -k 10 120 env "$@" python3 tools/q8_decode.py --bf16 --rows 1 2>&1 | tail -1; }
echo "unfused:        $(run MX_UNUSED=1)"
echo "poll 20:        $(run MX_ATTN_O=1 MX_AO_POLL=20)"
echo "poll 100:       $(run MX_ATTN_O=1 MX_AO_POLL=100)"
echo "poll 20 nopre:  $(run MX_ATTN_O=1 MX_AO_POLL=20 MX_AO_NOPREFETCH=1)"
echo "unfused:        $(run MX_UNUSED=1)"
