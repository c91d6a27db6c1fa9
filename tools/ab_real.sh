#!/bin/bash
# A/B of library variants on the real-env step (tools/bench_real_env.py, E envs at 324 x 450):
#   bash tools/ab_real.sh OUT_DIR lib1.so [lib2.so ...]      (run through gpurun)
# the real-env GPU tests on the default library first, then alternating timed runs.
OUT=${1:-gpurun_out/abr}; shift
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_real_env.py \
    tests/test_gpu_real_bids.py tests/test_gpu_filtered.py > "$OUT/tests.log" 2>&1 \
    || { echo "real tests failed"; tail -5 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
for rep in $(seq ${AB_REPS:-2}); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python tools/bench_real_env.py --envs ${REAL_ENVS:-512} --steps 20 --cpu 0 > "$OUT/r.json" 2>&1 \
        || { echo "bench failed for $lib"; tail -5 "$OUT/r.json"; exit 1; }
    python3 -c "
import json
d = json.loads([l for l in open('$OUT/r.json') if l.startswith('{')][-1])
print('$lib', d['value'], d['step_ms'], d['roofline']['frac'])"
  done
done
