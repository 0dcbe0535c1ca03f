# gate/up geometry A/B at batch 1 (graph replay): register-held B fragments, 1 work-group per CU
# (default) vs LDS-read fragments at 64 VGPRs (2 work-groups per CU) with 7/4/2/1 tiles per group
export TMPDIR=/tmp
set -e
for i in 1 2; do
  echo "base   $(MX_NO_PERS=1 timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1)"
  echo "u8     $(timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1)"
  for t in 7 4 2 1; do
    echo "xl_t$t  $(MX_PERS_TPW=$t timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 1)"
  done
done
