#!/bin/bash
# Bench A/B on one box: fused rollout kernel (--fused-rollout 2) vs separate step + select
# launches (0), alternating, at configs[2] (64x64); "256" adds configs[4] (256x256 dense).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
rocm-smi --showclocks 2>/dev/null | grep -i "sclk\|mclk" | head -4
for f in 2 0 2 0 2 0; do timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --fused-rollout $f || exit 1; done
if [ "$1" = 256 ]; then
  for f in 2 0 2 0; do timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --secondary 0 --fused-rollout $f || exit 1; done
fi
rocm-smi --showclocks 2>/dev/null | grep -i "sclk\|mclk" | head -4
