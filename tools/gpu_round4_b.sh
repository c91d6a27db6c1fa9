#!/bin/bash
# Round-4 checks of the REDA step_q schedule (asg_step_forward + asg_sap_select_into), then
# the SAP bench leg on it:  bash tools/gpu_round4_b.sh OUT_DIR
set -o pipefail
OUT=${1:-gpurun_out/r4b}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step_q.py \
    tests/test_gpu_runner.py -k "step_q or step_forward or select_into or yaml" \
    > "$OUT/tests.log" 2>&1 || { echo "FAILED tests"; tail -60 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 40 --warmup 10 \
    > "$OUT/bench_sap.log" 2>&1 || { echo "FAILED bench"; tail -20 "$OUT/bench_sap.log"; exit 1; }
python3 - "$OUT/bench_sap.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", d["value"], "ms/step", d["ms_per_step"], json.dumps(d["kernels_ms"]))
print("roofline", json.dumps(d["roofline"])[:400])
PY
