#!/bin/bash
# GPU validation on one MI355X (run through gpurun from the repo root):
#   tools/gpu_check.sh OUT_DIR [PYTEST_K]
# 1. the GPU tests selected by PYTEST_K (all when empty), 2. the whole GPU suite (skipped
# when PYTEST_K is "only"), 3. smoke(), 4. the driver's bench command.  Every step has its
# own time limit; a step that times out, aborts or faults (exit 124 / 134 / 137 / 139) ends
# the script, an ordinary test failure does not stop the later steps.
OUT=${1:-gpurun_out/check}
K=${2:-}
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit "$1";; esac; }
if [ -n "$K" ] && [ "$K" != "all" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" \
        > "$OUT/sel_tests.log" 2>&1
    rc=$?; echo "selected tests rc=$rc"; tail -3 "$OUT/sel_tests.log"; fatal $rc selected-tests
fi
if [ "$K" != "only" ]; then
    timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1
    rc=$?; echo "gpu tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; fatal $rc gpu-tests
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; fatal $rc smoke
    timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1
    rc=$?; echo "bench rc=$rc"; tail -c 4000 "$OUT/bench.log"; fatal $rc bench
fi
exit 0
