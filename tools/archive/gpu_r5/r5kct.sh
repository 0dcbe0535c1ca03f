# A/B of the bf16 32-row gate/up GEMV's activation-chunk depth (MX_WIDE_KCT 4 / 8): kernel time, whole
# 32-sequence decode step (bench.py main line), and the -m gpu suite at 8
# (record of a finished A/B: the switch it sets was removed from the engine afterwards -- see git log for the build it ran on)
set -o pipefail
O=gpurun_out/r5kct; mkdir -p $O
for r in 1 2; do for k in 4 8; do
  MX_WIDE_KCT=$k MX_WIDE_KCT_SLAB=$k timeout -k 10 200 python -u tools/step_probe.py --M 32 --kinds 0,1,2,3 > $O/s$k$r.log 2>&1 || { tail -20 $O/s$k$r.log; exit 1; }
  echo "kct $k run $r $(grep -o '{"M".*' $O/s$k$r.log | cut -c1-400)"
done; done
for k in 4 8 48; do
  MX_WIDE_KCT=${k:0:1} MX_WIDE_KCT_SLAB=${k: -1} timeout -k 10 400 python -u bench.py --no-cpu-baseline --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --geometry-steps 0 --serve-requests 0 --prefill-prompts 0 --tiny-tokens 0 > $O/b$k.json 2> $O/b$k.err || { tail -20 $O/b$k.err; exit 1; }
  echo "kct $k bench $(python3 -c "import json; d=json.loads(open('$O/b$k.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['us_per_launch'], d['roofline']['frac'])")"
done
MX_WIDE_KCT=8 MX_WIDE_KCT_SLAB=8 timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest8.log 2>&1 || { tail -30 $O/pytest8.log; exit 1; }
tail -1 $O/pytest8.log
