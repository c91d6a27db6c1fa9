#!/bin/bash
# Round-4 checks of the new paths (run through gpurun from the repo root):
#   bash tools/gpu_round4_a.sh OUT_DIR
set -o pipefail
OUT=${1:-gpurun_out/r4a}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sap.py \
    tests/test_gpu_fused_rollout.py tests/test_gpu_runner.py tests/test_gpu_timed_path.py \
    > "$OUT/tests.log" 2>&1 || { echo "FAILED tests"; tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
