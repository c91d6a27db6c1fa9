#!/bin/bash
# Does the timed region of the driver's command (20 steps after 5 warmup steps, right after the
# 15-s CPU baseline leaves the GPU idle) run slower than a longer run on the same box?
#   bash tools/warm_probe.sh OUT   (through gpurun)
OUT=${1:-gpurun_out/warm}; mkdir -p "$OUT"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --secondary 0 "$@" > "$OUT/$name.json" 2>&1 || { echo "FAILED $name"; tail -3 "$OUT/$name.json"; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][-1]); k = d['kernels_ms']
print('$name', d['steps'], d['warmup'], d['value'], d['ms_per_step'], k.get('fused_rollout_per_step'))"
}
for rep in 1 2; do
  run driver_cmd --steps 20 --warmup 5
  run no_cpu --cpu-baseline 0 --steps 20 --warmup 5
  run long --cpu-baseline 0 --steps 60 --warmup 20
done
