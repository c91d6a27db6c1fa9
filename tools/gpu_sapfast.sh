#!/bin/bash
# The certified SAP fast path: its parity tests, the SAP/LSA/HAA/runner parity tests, then the
# bench's SAP leg against the exact-only library (build/lib_exact.so, -DASG_SAP_FAST=0):
#   bash tools/gpu_sapfast.sh OUT_DIR
set -o pipefail
OUT=${1:-gpurun_out/sapfast}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sap.py tests/test_gpu_parity.py tests/test_gpu_learner.py \
    tests/test_gpu_step_q.py > "$OUT/tests.log" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -20; tail -5 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do
  for lib in default build/lib_exact.so; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    tag=$(basename "$lib" .so)
    timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 \
        > "$OUT/bench_${tag}_$rep.log" 2>&1 || { echo "FAILED bench $lib"; tail -5 "$OUT/bench_${tag}_$rep.log"; exit 1; }
    python3 - "$OUT/bench_${tag}_$rep.log" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline_lsa"]
print(sys.argv[2], "value", d["value"], "sap_kernel_ms", r["kernel_ms"], "steps fast/exact", r.get("path_steps_fast"),
      r.get("path_steps_exact"), "exact problems", r.get("problems_on_exact_solver"), json.dumps(d["kernels_ms"]))
PY
  done
done
# host-side profile of the SAP leg (where the per-episode first selection spends its time)
timeout -k 10 300 python -m cProfile -o "$OUT/sap.prof" bench.py --selector sap --cpu-baseline 0 --secondary 0 \
    --steps 40 --warmup 5 > "$OUT/cprof_bench.log" 2>&1 || { echo "FAILED cprofile"; exit 1; }
python -c "import pstats; pstats.Stats('$OUT/sap.prof').sort_stats('tottime').print_stats(20)" > "$OUT/cprof.txt"
