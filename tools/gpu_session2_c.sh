#!/bin/bash
# session-2 checks: SAP / step_q tests, the SAP A/B (previous library, staging only), the
# same-seed mode's kernel statistics, then the driver's bench command
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out/r4_compat7 gpurun_out/r4_s2_bench3
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sap.py tests/test_gpu_step_q.py > gpurun_out/r4_s2_bench3/tests.log 2>&1 || { echo "FAILED tests"; tail -20 gpurun_out/r4_s2_bench3/tests.log; exit 1; }
tail -1 gpurun_out/r4_s2_bench3/tests.log
REPS=2 bash tools/ab_sap_bench.sh gpurun_out/r4_s2_sapab9 build/lib_prev.so build/lib_stageonly.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_compat7/kt -o run -- python3 bench.py --rng mt19937 --cpu-baseline 0 --secondary 0 --steps 40 --warmup 5 > gpurun_out/r4_compat7/b.log 2>&1 || { echo "FAILED compat profile"; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_s2_bench3/bench.log 2>&1 || { echo "FAILED bench"; exit 1; }
echo done
