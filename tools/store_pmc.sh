#!/bin/bash
# Store-path counters of the episode kernel (run through gpurun from the repo root):
#   bash tools/store_pmc.sh OUT_DIR
# one SQ pass per config (2: 64 x 64, 4: 256 x 256) over one reset + 20-step launch.
set -o pipefail
OUT=${1:-gpurun_out/store_pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P="SQ_INST_CYCLES_VMEM_WR SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"
for cfg in 2 4; do
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/c$cfg" -o run -- python3 bench.py --cpu-baseline 0 \
      --secondary 0 --steps 20 --warmup 0 --config $cfg > "$OUT/c$cfg.log" 2>&1 || { echo "FAILED c$cfg"; tail -5 "$OUT/c$cfg.log"; exit 1; }
done
echo done
