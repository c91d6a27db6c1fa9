#!/bin/bash
# The driver's window on the GPU's clock ramp: per-launch durations of the episode kernel in the
# driver's command (bench.py --steps 20 --warmup 5, no secondary legs) and in a longer window,
# from rocprofv3 kernel traces (GPU box, repo root):  bash tools/ramp_trace.sh OUT_DIR
set -o pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for w in "20:5" "60:20"; do
  s=${w%:*}; wu=${w#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$s" -o run -- \
      python3 bench.py --cpu-baseline 0 --secondary 0 --steps $s --warmup $wu > "$OUT/log_$s" 2>&1 \
      || { echo "FAILED $w"; tail -5 "$OUT/log_$s"; exit 1; }
  python3 - "$OUT/kt_$s" "$s" "$wu" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "rollout_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
print(f"--steps {sys.argv[2]} --warmup {sys.argv[3]}: episode-kernel launches (start ms after the first, duration ms)")
for r in rows:
    print(f"  {(int(r['Start_Timestamp']) - t0) / 1e6:9.3f}  {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:8.4f}")
PY
done
