#!/bin/bash
# Bench A/B across library variants (whole bench lines, fused and split schedules, SAP leg),
# after the bit-exactness suites on the in-tree library:  bash tools/ab_bench.sh [lib ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_rollout.py tests/test_gpu_sap.py tests/test_gpu_runner.py > gpurun_out/ab_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    for f in 1 0; do
      timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --fused-rollout $f > gpurun_out/ab_b.json 2>&1 || exit 1
      python3 -c "
import json
for l in open('gpurun_out/ab_b.json'):
    if l.startswith('{'):
        d = json.loads(l); k = d['kernels_ms']
        print('$lib fused=$f', d['value'], d['ms_per_step'], k['fused_step_select'], k['env_step'], k['select'])"
    done
    timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 > gpurun_out/ab_b.json 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/ab_b.json'):
    if l.startswith('{'):
        d = json.loads(l); print('$lib sap', d['value'], d['roofline_lsa']['kernel_ms'])"
  done
done
