#!/bin/bash
# A/B of fused-rollout library variants (tools/ab_rollout.py per library, twice), after the
# fused-rollout bit-identity tests on the in-tree library:  bash tools/ab_rollout.sh [lib ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_rollout.py > gpurun_out/fr_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then timeout -k 10 120 python tools/ab_rollout.py || exit 1
    else ASG_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/ab_rollout.py || exit 1; fi
  done
done
