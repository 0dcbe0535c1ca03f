#!/bin/bash
# Submit a command to the GPU box via gpurun.  Re-submits ONLY when gpurun reports
# status=transient or no box (exit 3): nothing of the command ran, nothing charged.  Honours the
# back-off gpurun asks for ("retry in Ns").  A command that ran and failed is never retried.
#   tools/gpu.sh <timeout_s> '<command>'
python3 llama-p2p_amd/build.py > /dev/null || { echo "[gpu.sh] build failed" >&2; exit 1; }
T=${1:-600}
shift
LOG=$(mktemp)
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1 | tee "$LOG"
  rc=${PIPESTATUS[0]}
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" = "transient" ] || [ $rc -eq 3 ]; then
    wait_s=$(grep -o 'retry in [0-9]*s' "$LOG" | tail -1 | grep -o '[0-9]*')
    wait_s=${wait_s:-45}
    echo "[gpu.sh] transient/no box (attempt $attempt); waiting $((wait_s + 10))s before re-submitting" >&2
    sleep $((wait_s + 10))
    continue
  fi
  rm -f "$LOG"
  exit $rc
done
rm -f "$LOG"
exit $rc
