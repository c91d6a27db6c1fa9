#!/bin/bash
# Where the same-seed reset's draw kernel spends its time: kernel traces of the compat leg
# (bench.py --rng mt19937) with the timing-only builds of tools' ASG_MT_XSKIP bits (WRONG results):
#   for v in 1 2 4; do python -m marl_sap_amd.build --out build/mtx$v.so -DASG_TIMING_EXPERIMENTS \
#       -DASG_MT_XSKIP=$v; done        (CPU side), then on the GPU box: bash tools/mt_timing.sh OUT_DIR
set -o pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in default 1 2 4; do
  if [ "$v" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/build/mtx$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$v" -o run -- \
      python3 bench.py --cpu-baseline 0 --secondary 0 --rng mt19937 --steps 40 --warmup 10 > "$OUT/log_$v" 2>&1 \
      || { echo "FAILED $v"; tail -5 "$OUT/log_$v"; exit 1; }
  python3 - "$OUT/kt_$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in csv.DictReader(open(f)):
    if "mt_reset" in x["Name"] or "mt_table" in x["Name"]:
        print(sys.argv[2], x["Name"][:40], x["Calls"], "avg ms", round(float(x["AverageNs"]) / 1e6, 4),
              "min ms", round(float(x["MinNs"]) / 1e6, 4))
PY
done
