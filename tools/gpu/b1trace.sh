# batch-1 bf16 decode: graph timing, then an eager rocprofv3 kernel trace summarised per kernel/grid
export TMPDIR=/tmp
set -e
timeout -k 10 120 python3 tools/q8_decode.py --model ${MODEL:-llama3-8b} --rows ${ROWS:-1} --bf16
MX_NO_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b1t -o b1t -- python3 tools/q8_decode.py --model ${MODEL:-llama3-8b} --bf16 --rows ${ROWS:-1} --steps 32 > gpurun_out/b1t.log 2>&1
grep rows gpurun_out/b1t.log
python3 profiles/analyze_trace.py $(ls gpurun_out/b1t/*/b1t_kernel_trace.csv gpurun_out/b1t/b1t_kernel_trace.csv 2>/dev/null | head -1) --last 7000 > gpurun_out/b1t_summary.txt
cat gpurun_out/b1t_summary.txt
