# batch-1 bf16 decode: graph timing, then an eager rocprofv3 kernel trace (current kernels)
export TMPDIR=/tmp
set -e
timeout -k 10 120 python3 tools/q8_decode.py --rows 1 --bf16
MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/b1n -o b1n -- python3 tools/q8_decode.py --bf16 --rows 1 --steps 32 > gpurun_out/b1n.log 2>&1
grep rows gpurun_out/b1n.log
