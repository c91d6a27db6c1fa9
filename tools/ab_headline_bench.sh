#!/bin/bash
# headline (configs[2]) bench A/B, 60 steps after 20 across library variants:
#   bash tools/ab_headline_bench.sh OUT_DIR lib1.so [lib2.so ...]   (REPS, default 2)
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in $(seq 1 ${REPS:-2}); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    tag=$(basename "$lib" .so)
    timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --steps 60 --warmup 20 \
        > "$OUT/bench_${tag}_$rep.log" 2>&1 || { echo "FAILED bench $lib"; tail -5 "$OUT/bench_${tag}_$rep.log"; exit 1; }
    python3 - "$OUT/bench_${tag}_$rep.log" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:28s} value {d['value']:.4g} ms/step {d['ms_per_step']} kernel {d['kernels_ms']['fused_rollout_per_step']} frac {d['roofline']['frac']}")
PY
  done
done
