#!/bin/bash
# SAP-leg A/B across library variants, no tests (scheduling / occupancy variants of the same
# solver):  bash tools/ab_sap_bench.sh OUT_DIR lib1.so [lib2.so ...]   (REPS, default 2)
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in $(seq 1 ${REPS:-2}); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    tag=$(basename "$lib" .so)
    timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 \
        > "$OUT/bench_${tag}_$rep.log" 2>&1 || { echo "FAILED bench $lib"; tail -5 "$OUT/bench_${tag}_$rep.log"; exit 1; }
    python3 - "$OUT/bench_${tag}_$rep.log" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d.get("roofline_lsa") or {}
print(f"{sys.argv[2]:28s} value {d['value']:.4g} sap_kernel_ms {r.get('kernel_ms', d['kernels_ms'].get('sap_select'))} "
      f"cyc/step {r.get('cycles_per_step_per_simd')} exact_problems {r.get('problems_on_exact_solver')}")
PY
  done
done
