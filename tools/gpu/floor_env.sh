#!/bin/bash
# Kernel-boundary floor (tools/phase_probe bare mode, 256 and 1024 groups) under HIP runtime settings
#   tools/gpu/floor_env.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
for cfg in "base" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1"; do
  if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
  env $e timeout -k 10 60 ./tools/phase_probe bare > $OUT/floor_$cfg.log 2>&1 || { tail -5 $OUT/floor_$cfg.log; exit 1; }
  echo "$cfg: $(grep -E '"bare_groups": (256|1024), "threads": 1024' $OUT/floor_$cfg.log | tr '\n' ' ')"
done
