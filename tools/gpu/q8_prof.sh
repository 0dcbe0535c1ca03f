# Q8_0 batch-1 decode: graph timing, then an eager rocprofv3 kernel trace
export TMPDIR=/tmp
set -e
timeout -k 10 120 python3 tools/q8_decode.py --rows 1
MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/q8p -o q8p -- python3 tools/q8_decode.py --rows 1 --steps 32 > gpurun_out/q8p.log 2>&1
cat gpurun_out/q8p.log
