#!/bin/bash
# A/B of fused-rollout library variants at configs[4]'s shape (256x256, E = 2048, L = 3,
# T = 20; tools/ab_rollout.py per library, twice):  bash tools/ab_rollout_256.sh [lib ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then timeout -k 10 120 python tools/ab_rollout.py 2048 256 256 3 20 || exit 1
    else ASG_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/ab_rollout.py 2048 256 256 3 20 || exit 1; fi
  done
done
