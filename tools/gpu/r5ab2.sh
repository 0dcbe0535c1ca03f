set -o pipefail
timeout -k 10 200 python -u tools/step_probe.py --kinds 1,3,15,16,8,9,10,13,14 > gpurun_out/r5ab2_probe.json 2>&1 || exit 1
cat gpurun_out/r5ab2_probe.json
bash tools/gpu/ab_env.sh r5ab2 "- MX_WIDE_KS=1 MX_WIDE_KS=1,MX_WIDE_NOL=1" "--steps 64"
