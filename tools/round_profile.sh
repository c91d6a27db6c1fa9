#!/bin/bash
# Round-end evidence on one MI355X (run through gpurun from the repo root):
#   GPU tests, smoke(), the default bench line, rocprofv3 kernel statistics of the bench,
#   and separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters) for the step and agent
#   kernels.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -q > "$OUT/gpu_tests.log" 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --cpu-baseline 0 > "$OUT/kt.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 > "$OUT/write.log" 2>&1 &&
timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 > "$OUT/bench_sap.log" 2>&1 &&
timeout -k 10 300 python tools/bench_lsa.py > "$OUT/bench_lsa.json" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_sap" -o run -- python3 bench.py --selector sap --cpu-baseline 0 --steps 20 --warmup 5 > "$OUT/kt_sap.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run -- python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 > "$OUT/sq.log" 2>&1
