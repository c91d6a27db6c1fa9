#!/bin/bash
# round-5 GPU session step (gpurun, repo root): selected GPU tests, then an A/B of library
# variants on the episode kernel, then the SAP / REDA bench legs.  Each step has its own limit.
#   bash tools/gpu_r5.sh OUT_DIR "PYTEST_K" [lib.so ...]
OUT=${1:?out}; K=${2:-}; shift 2
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit "$1";; esac; }
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > "$OUT/sel.log" 2>&1
  rc=$?; echo "selected tests rc=$rc"; grep -E "passed|failed" "$OUT/sel.log" | tail -3; fatal $rc tests
fi
if [ $# -gt 0 ]; then
  AB_REPS=${AB_REPS:-3} timeout -k 10 900 bash tools/ab_episode.sh "$OUT/ab" "$@" > "$OUT/ab.log" 2>&1
  rc=$?; echo "ab rc=$rc"; tail -$((3 * (${AB_REPS:-3}) * ($# + 1))) "$OUT/ab.log"; fatal $rc ab
fi
if [ -n "$BENCH_SAP" ]; then
  timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 40 --warmup 20 > "$OUT/bench_sap.log" 2>&1
  rc=$?; echo "bench sap rc=$rc"; fatal $rc bench_sap
  python3 - "$OUT/bench_sap.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("sap", d["value"], d["ms_per_step"], d["kernels_ms"], (d.get("roofline_lsa") or {}).get("path_steps_per_launch"))
PY
fi
exit 0
