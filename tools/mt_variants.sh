#!/bin/bash
# The same-seed reset's draw kernel (mt_reset_kernel) time per library variant: kernel traces of
# the compat leg (bench.py --rng mt19937), min / avg over the window's resets.
#   bash tools/mt_variants.sh OUT_DIR lib1.so [lib2.so ...]      ("default" = the in-tree library)
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in default "$@"; do
  tag=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$tag" -o run -- \
      python3 bench.py --cpu-baseline 0 --secondary 0 --rng mt19937 --steps 40 --warmup 10 > "$OUT/log_$tag" 2>&1 \
      || { echo "FAILED $lib"; tail -5 "$OUT/log_$tag"; exit 1; }
  python3 - "$OUT/kt_$tag" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in csv.DictReader(open(f)):
    if "mt_reset" in x["Name"] or "mt_table" in x["Name"] or "rollout_kernel" in x["Name"]:
        print(f"{sys.argv[2]:10s}", x["Name"][:40], x["Calls"], "avg ms", round(float(x["AverageNs"]) / 1e6, 4),
              "min ms", round(float(x["MinNs"]) / 1e6, 4))
PY
done
