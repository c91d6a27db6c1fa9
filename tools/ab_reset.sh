#!/bin/bash
# A/B of the fused episode reset (bench.py --fuse-reset 1 vs 0) on one box (run through gpurun):
#   bash tools/ab_reset.sh OUT_DIR
OUT=${1:-gpurun_out/ab_reset}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for fr in 1 0; do
    timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --steps 40 --warmup 20 --fuse-reset $fr \
        > "$OUT/b.json" 2>&1 || { echo "bench failed"; tail -5 "$OUT/b.json"; exit 1; }
    python3 -c "
import json
for l in open('$OUT/b.json'):
    if l.startswith('{'):
        d = json.loads(l); k = d['kernels_ms']
        print('fuse_reset=$fr', d['value'], d['ms_per_step'], k.get('fused_rollout_per_step'))"
  done
done
