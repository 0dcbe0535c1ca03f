#!/bin/bash
# Submit a command to the GPU box via gpurun.  Re-submits ONLY when gpurun reports
# status=transient (the box failed while being prepared: nothing of the command ran,
# nothing charged).  A command that ran and failed is never retried.
#   tools/gpu.sh <timeout_s> '<command>'
python3 llama-p2p_amd/build.py > /dev/null || { echo "[gpu.sh] build failed" >&2; exit 1; }
T=${1:-600}
shift
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" = "transient" ] || [ $rc -eq 3 ]; then
    echo "[gpu.sh] transient/no box (attempt $attempt); waiting before re-submitting" >&2
    sleep 30
    continue
  fi
  exit $rc
done
exit $rc
