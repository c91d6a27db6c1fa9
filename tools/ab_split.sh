#!/bin/bash
# A/B of library variants on the split schedule (env step + agent/select launches) and the
# episode schedule, after the agent / fused-rollout identity tests:  bash tools/ab_split.sh [lib ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_agent.py tests/test_gpu_fused_rollout.py tests/test_gpu_runner.py ${AB_TESTS:-} > gpurun_out/ab_split_tests.log 2>&1 || { tail -5 gpurun_out/ab_split_tests.log; exit 1; }
tail -1 gpurun_out/ab_split_tests.log
for rep in 1 2 3; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    for f in 1 0; do
      timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --fused-rollout $f --steps 40 --warmup 20 > gpurun_out/ab_s.json 2>&1 || exit 1
      python3 -c "
import json
for l in open('gpurun_out/ab_s.json'):
    if l.startswith('{'):
        d = json.loads(l); k = d['kernels_ms']
        print('$lib fused=$f', d['value'], d['ms_per_step'], k.get('fused_rollout_per_step'), k.get('env_step'), k.get('select'))"
    done
  done
done
