set -o pipefail
VARIANTS="dw dw4" QUANT=q4_0 TESTS="tests/test_q4_0_gpu.py" KINDS=2 bash tools/gpu/r5q4w.sh && \
VARIANTS="base kq8" QUANT=q4_k_m TESTS="tests/test_kquants_gpu.py" KINDS=2,4 bash tools/gpu/r5q4w.sh
