# 32-row bf16 decode: graph timing, then an eager rocprofv3 kernel trace
export TMPDIR=/tmp
set -e
timeout -k 10 120 python3 tools/q8_decode.py --bf16 --rows 32 | tail -1
MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/m32 -o m32 -- python3 tools/q8_decode.py --bf16 --rows 32 --steps 32 > gpurun_out/m32.log 2>&1
grep rows gpurun_out/m32.log
