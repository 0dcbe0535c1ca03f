#!/bin/bash
# Round 6: generic-shape paths -- the Llama-2-7B geometry oracle test, batch invariance, and the bench's
# geometry section (8B sections trimmed).
set -o pipefail
TAG=${1:-r6g}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_batch_invariance_gpu.py "tests/test_fulldepth_stages_gpu.py::test_llama2_7b_geometry_sampled_layers_vs_oracle" tests/test_engine_gpu.py -x -v -s --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
grep -E "Llama-2|passed|failed" $OUT/pytest.log | tail -4
timeout -k 10 500 python -u bench.py --batch1-steps 32 --tiny-tokens 64 --prefill-prompts 0 --q8-steps 0 --kq-steps 0 --q40-steps 0 --big-steps 0 --serve-requests 0 --no-cpu-baseline "$@" > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['step_hbm_frac'], d['batch1']['hbm_frac'], d['tinyllama']['batch1']['hbm_frac'], json.dumps(d.get('llama2_7b_geometry')))"
