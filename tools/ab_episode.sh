#!/bin/bash
# A/B of library variants on the whole-episode fused rollout (bench headline schedule):
#   bash tools/ab_episode.sh OUT_DIR lib1.so [lib2.so ...]      (run through gpurun)
# First the fused-vs-split bit-identity tests on every variant (a variant must not change
# results), then alternating bench runs (2 timed episodes each), printing the kernel time per
# step.  Every step has its own time limit; the script stops at the first failure.
OUT=${1:-gpurun_out/ab}; shift
mkdir -p "$OUT"
for lib in default "$@"; do
  case "$lib" in *timing*) continue;; esac   # timing-only builds (wrong results) skip the identity tests
  if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_rollout.py \
      -k "bit_identical and (64-64-6 or 20-25 or 256-256) or chunks" > "$OUT/tests_$(basename $lib).log" 2>&1 \
      || { echo "tests failed for $lib"; tail -5 "$OUT/tests_$(basename $lib).log"; exit 1; }
done
for rep in $(seq ${AB_REPS:-3}); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    for cfg in "${AB_CONFIGS:-2}"; do
      timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --steps 40 --warmup 20 --config $cfg \
          ${AB_EXTRA:-} > "$OUT/b.json" 2>&1 || { echo "bench failed for $lib"; tail -5 "$OUT/b.json"; exit 1; }
      python3 -c "
import json
for l in open('$OUT/b.json'):
    if l.startswith('{'):
        d = json.loads(l); k = d['kernels_ms']
        print('$lib cfg=$cfg', d['value'], d['ms_per_step'], k.get('fused_rollout_per_step'))"
    done
  done
done
