#!/bin/bash
# A/B of the SAP selector kernel across library variants (build/*.so built with -D flags by
#   python -m marl_sap_amd.build --out build/lib_X.so -DFLAG=...):
#   bash tools/ab_sap_libs.sh OUT_DIR lib1.so [lib2.so ...]
# Each variant first passes the SAP parity tests (tests/test_gpu_sap.py) on itself, then the
# bench's SAP leg runs REPS times per variant, interleaved (sap_select kernel ms, cycles/step).
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in default "$@"; do
  if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
  tag=$(basename "$lib" .so)
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sap.py tests/test_gpu_parity.py \
      -k "sap or lsa or haa or eps0" > "$OUT/tests_$tag.log" 2>&1 || { echo "FAILED tests $lib"; tail -20 "$OUT/tests_$tag.log"; exit 1; }
  echo "tests ok $lib: $(tail -1 "$OUT/tests_$tag.log")"
done
for rep in $(seq 1 ${REPS:-2}); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
    tag=$(basename "$lib" .so)
    timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 \
        > "$OUT/bench_${tag}_$rep.log" 2>&1 || { echo "FAILED bench $lib"; tail -5 "$OUT/bench_${tag}_$rep.log"; exit 1; }
    python3 - "$OUT/bench_${tag}_$rep.log" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline_lsa"]
print(sys.argv[2], "sap_kernel_ms", r["kernel_ms"], "cyc/step/simd", r["cycles_per_step_per_simd"], "value", d["value"])
PY
  done
done
