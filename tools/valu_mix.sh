#!/bin/bash
# VALU instruction mix of the episode kernel (run through gpurun from the repo root):
#   bash tools/valu_mix.sh OUT_DIR
# two SQ passes over one reset + 20-step launch (configs[2]); every step has its own limit.
set -o pipefail
OUT=${1:-gpurun_out/valu_mix}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --cpu-baseline 0 --secondary 0 --steps 20 --warmup 0"
P1="SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_MFMA SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
timeout -k 10 300 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/p1" -o run -- python3 $B > "$OUT/p1.log" 2>&1 || { echo "FAILED p1"; tail -5 "$OUT/p1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/p2" -o run -- python3 $B > "$OUT/p2.log" 2>&1 || { echo "FAILED p2"; tail -5 "$OUT/p2.log"; exit 1; }
echo done
