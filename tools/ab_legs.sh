#!/bin/bash
# A/B of library variants on one bench configuration, printing value, ms/step and every
# kernels_ms entry (gpurun, repo root):
#   AB_ARGS="--selector sap" AB_REPS=3 bash tools/ab_legs.sh OUT_DIR lib1.so [lib2.so ...]
# "default" = the in-tree library.  Each bench run has its own time limit.
OUT=${1:?out}; shift
mkdir -p "$OUT"
for rep in $(seq ${AB_REPS:-2}); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --steps ${AB_STEPS:-40} --warmup 20 ${AB_ARGS:-} \
        > "$OUT/b.json" 2>&1 || { echo "bench failed for $lib"; tail -5 "$OUT/b.json"; exit 1; }
    python3 - "$OUT/b.json" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = {a: b for a, b in d["kernels_ms"].items() if isinstance(b, float)}
print(f"{sys.argv[2]:26s} {d['value']:.4g} {d['ms_per_step']} {k}")
PY
  done
done
