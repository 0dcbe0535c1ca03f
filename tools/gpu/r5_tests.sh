#!/bin/bash
# full -m gpu suite + smoke, then per-kernel probes of the 32-row layer
set -o pipefail
O=gpurun_out/${1:-r5t}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python -u tools/step_probe.py > $O/probe_wide.json 2> $O/probe_wide.err || exit 1
MX_NO_WIDE=1 timeout -k 10 120 python -u tools/step_probe.py --kinds 0,1,2,3,10 > $O/probe_nowide.json 2> $O/probe_nowide.err || exit 1
cat $O/probe_*.json
