#!/bin/bash
# Same-seed (MT19937) mode A/B across library variants: the headline workload with --rng mt19937
# (asg_reset's draws + table kernel, then the episode kernel), then a kernel-trace of each
# library:  bash tools/ab_compat.sh OUT_DIR lib1.so [lib2.so ...]   (REPS, default 2)
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in $(seq 1 ${REPS:-2}); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    tag=$(basename "$lib" .so)
    timeout -k 10 300 python bench.py --rng mt19937 --cpu-baseline 0 --secondary 0 --steps 40 --warmup 20 \
        > "$OUT/bench_${tag}_$rep.log" 2>&1 || { echo "FAILED bench $lib"; tail -5 "$OUT/bench_${tag}_$rep.log"; exit 1; }
    python3 - "$OUT/bench_${tag}_$rep.log" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:28s} value {d['value']:.4g} ms_per_step {d['ms_per_step']} kernels {d.get('kernels_ms')}")
PY
  done
done
for lib in default "$@"; do
  if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
  tag=$(basename "$lib" .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$tag" -o run -- python3 bench.py \
      --rng mt19937 --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 > "$OUT/prof_$tag.log" 2>&1 \
      || { echo "FAILED profile $lib"; exit 1; }
  f=$(find "$OUT/prof_$tag" -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; [ -n "$f" ] && grep -E 'mt_|reset_kernel|rollout_kernel' "$f" | cut -c1-200
done
exit 0
