#!/bin/bash
# PMC passes over tools/ab_rollout.py (fused rollout kernel vs step + select), per library:
#   bash tools/pmc_rollout.sh OUT [lib ...]   ("default" = the in-tree library)
set -o pipefail
OUT=${1:-gpurun_out/pmc_rollout}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/$tag-p1" -o run -- python3 tools/ab_rollout.py 16384 64 64 3 20 1 4 > "$OUT/$tag-p1.log" 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/$tag-p2" -o run -- python3 tools/ab_rollout.py 16384 64 64 3 20 1 4 > "$OUT/$tag-p2.log" 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$tag-f" -o run -- python3 tools/ab_rollout.py 16384 64 64 3 20 1 4 > "$OUT/$tag-f.log" 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$tag-w" -o run -- python3 tools/ab_rollout.py 16384 64 64 3 20 1 4 > "$OUT/$tag-w.log" 2>&1 || exit 1
done
