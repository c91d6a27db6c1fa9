#!/bin/bash
# A/B of the SAP selector kernel (bench.py --selector sap: lsa_ms) across library variants,
# after the LSA / SAP parity tests on the in-tree library:  bash tools/ab_sap.sh [lib ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sap.py tests/test_gpu_parity.py tests/test_gpu_filtered.py tests/test_gpu_real_env.py > gpurun_out/sap_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 > gpurun_out/ab_sap.json 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/ab_sap.json'):
    if l.startswith('{'):
        d = json.loads(l); r = d['roofline_lsa']
        print('$lib', 'lsa_ms', r['kernel_ms'], 'cyc/step', r['cycles_per_step_per_simd'], 'value', d['value'])"
  done
done
