#!/bin/bash
# SAP selector: parity of the multi-problem-per-wave kernels, then the bench's SAP leg per
# setting of asg_sap_slots (0: one problem per wave, static grid; 1..3: persistent waves with
# that many interleaved problems).  Run through gpurun from the repo root:
#   bash tools/ab_sap_slots.sh OUT_DIR
set -o pipefail
OUT=${1:-gpurun_out/sap_ab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sap.py \
    > "$OUT/sap_tests.log" 2>&1 || { echo "FAILED tests"; tail -30 "$OUT/sap_tests.log"; exit 1; }
echo "tests ok"
for s in ${SLOTS:-0 1 2 3}; do
  ASG_SAP_SLOTS=$s timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 \
      --warmup 5 > "$OUT/bench_sap_slots$s.log" 2>&1 || { echo "FAILED slots $s"; tail -5 "$OUT/bench_sap_slots$s.log"; exit 1; }
  python - "$OUT/bench_sap_slots$s.log" $s <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
r = d.get("roofline_lsa") or {}
print("slots", sys.argv[2], "value", d["value"], "ms/step", d["ms_per_step"], "sap_kernel_ms", r.get("kernel_ms"),
      "cyc/step/simd", r.get("cycles_per_step_per_simd"), "steps", r.get("path_steps_per_launch"))
PY
done
