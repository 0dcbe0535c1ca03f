set -o pipefail
O=gpurun_out/r5attn; mkdir -p $O
MX_ATTN_TRACE=1 MX_PROF_FIN=1 timeout -k 10 200 python -u tools/attn_probe.py --rows 32 --pos 100,150,200,250 > $O/fin.json 2> $O/fin.trace || exit 1
MX_ATTN_TRACE=1 timeout -k 10 200 python -u tools/attn_probe.py --rows 32,1 --pos 150,250 > $O/nofin.json 2> $O/nofin.trace || exit 1
cat $O/fin.json $O/nofin.json; grep "attn trace" $O/fin.trace $O/nofin.trace
