#!/bin/bash
# Round-end evidence on one MI355X (run through gpurun from the repo root):
#   rocprofv3 kernel statistics of the default bench (configs[2]: the fused rollout kernel
#   asg_step_select) and of configs[4] (256x256 dense; its PMC passes on the split launches),
#   separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters) for the rollout, step and agent
#   kernels; the same for the split schedule (--fused-rollout 0) at configs[2]; the SAP leg.
#   Every GPU step has its own time limit; the chain stops at the first failure.
#   (GPU tests / smoke / the plain bench line run in their own call.)
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --cpu-baseline 0 --secondary 0"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 $B > "$OUT/kt.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $B --steps 20 --warmup 5 > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $B --steps 20 --warmup 5 > "$OUT/write.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/sq" -o run -- python3 $B --steps 20 --warmup 5 > "$OUT/sq.log" 2>&1 &&
timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --fused-rollout 0 > "$OUT/bench_split.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_split" -o run -- python3 $B --fused-rollout 0 > "$OUT/kt_split.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_split" -o run -- python3 $B --fused-rollout 0 --steps 20 --warmup 5 > "$OUT/fetch_split.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_split" -o run -- python3 $B --fused-rollout 0 --steps 20 --warmup 5 > "$OUT/write_split.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/sq_split" -o run -- python3 $B --fused-rollout 0 --steps 20 --warmup 5 > "$OUT/sq_split.log" 2>&1 &&
timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 > "$OUT/bench_256.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_256" -o run -- python3 $B --config 4 > "$OUT/kt_256.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_256" -o run -- python3 $B --config 4 --fused-rollout 0 --steps 20 --warmup 5 > "$OUT/fetch_256.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_256" -o run -- python3 $B --config 4 --fused-rollout 0 --steps 20 --warmup 5 > "$OUT/write_256.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_sap" -o run -- python3 $B --selector sap --steps 20 --warmup 5 > "$OUT/kt_sap.log" 2>&1 &&
timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 > "$OUT/bench_sap.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq_sap" -o run -- python3 $B --selector sap --steps 20 --warmup 5 > "$OUT/sq_sap.log" 2>&1 &&
timeout -k 10 300 python tools/bench_lsa.py > "$OUT/bench_lsa.json" 2>&1
