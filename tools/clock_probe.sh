#!/bin/bash
# Sample SCLK / power while the fused-rollout bench runs (box-to-box variance diagnosis).
cd "$GRAFT_REPO_ROOT" || exit 1
rocm-smi --showmaxpower 2>/dev/null | grep -i "power" | head -3
timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --steps 12000 --warmup 20 > gpurun_out/cp_bench.log 2>&1 &
pid=$!
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do sleep 2; rocm-smi --showclocks --showpower 2>/dev/null | grep -i "sclk\|power (" | head -3; done
wait $pid || exit 1
grep '^{' gpurun_out/cp_bench.log | cut -c1-200
