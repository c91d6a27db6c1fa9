#!/bin/bash
# SAP selector kernel time against resident waves per SIMD.  The cap is a compile-time knob
# (-DASG_SAP_LDS_PAD=<bytes> of unused dynamic LDS per 4-wave workgroup: 0 = the register
# limit, 5; 40960 = 4; 54000 = 3; 81920 = 2; 163840 = 1), so build the variants on the CPU first:
#   for p in 0 40960 54000 81920 163840; do
#     python -m marl_sap_amd.build --out build/sap_pad$p.so -DASG_SAP_LDS_PAD=$p; done
# then (GPU box, repo root): bash tools/sap_occupancy.sh OUT_DIR
set -o pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for pad in 0 40960 54000 81920 163840; do
  ASG_LIB_PATH=$PWD/build/sap_pad$pad.so timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 \
      --secondary 0 --steps 20 --warmup 5 > "$OUT/bench_pad$pad.log" 2>&1 || { echo "FAILED pad $pad"; tail -5 "$OUT/bench_pad$pad.log"; exit 1; }
  python3 - "$OUT/bench_pad$pad.log" $pad <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline_lsa"]
print("lds_pad", sys.argv[2], "sap_kernel_ms", r["kernel_ms"], "cyc/step/simd", r["cycles_per_step_per_simd"])
PY
done
