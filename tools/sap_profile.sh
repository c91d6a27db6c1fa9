#!/bin/bash
# SAP-leg LSA counters on one MI355X (run through gpurun from the repo root):
#   bash tools/sap_profile.sh OUT_DIR
# kernel statistics of the SAP bench, then one SQ pass (issue and wait cycles, scalar and
# vector instruction counts of sap_select_kernel).  Every GPU step has its own time limit.
set -o pipefail
OUT=${1:-gpurun_out/sap_prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 10 --warmup 3"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "counter list failed"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 $B \
    > "$OUT/kt.log" 2>&1 || { echo "FAILED kt"; tail -5 "$OUT/kt.log"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run -- python3 $B \
    > "$OUT/sq.log" 2>&1 || { echo "FAILED sq"; tail -5 "$OUT/sq.log"; exit 1; }
echo done
