#!/bin/bash
# round-6 GPU session step (gpurun, repo root).  Each GPU step has its own limit; the chain
# stops at the first fatal exit.
#   bash tools/gpu_r6.sh OUT_DIR STEPS...   STEPS from: tests[:K] bench compat_pmc bench_compat
OUT=${1:?out}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit "$1";; *) echo "exit $1 in $2";; esac; }
B="bench.py --cpu-baseline 0 --secondary 0"
for st in "$@"; do
  case "$st" in
    tests*)
      K=${TESTK:-}
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > "$OUT/tests.log" 2>&1
      rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" "$OUT/tests.log" | tail -5; fatal $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; fatal $rc smoke ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2> "$OUT/bench.err"
      rc=$?; echo "bench rc=$rc"; grep '^{' "$OUT/bench.log" | tail -1 | cut -c1-600; fatal $rc bench ;;
    bench_compat)
      timeout -k 10 300 python $B --rng mt19937 --steps 40 --warmup 20 > "$OUT/bench_compat.log" 2>&1
      rc=$?; echo "bench_compat rc=$rc"; grep '^{' "$OUT/bench_compat.log" | tail -1 | cut -c1-400; fatal $rc bench_compat ;;
    compat_pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_compat_$c" -o run -- python3 $B --rng mt19937 --steps 20 --warmup 0 > "$OUT/pmc_compat_$c.log" 2>&1
        rc=$?; echo "pmc $c rc=$rc"; fatal $rc pmc_$c
      done
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_compat" -o run -- python3 $B --rng mt19937 --steps 40 --warmup 20 > "$OUT/kt_compat.log" 2>&1
      rc=$?; echo "kt compat rc=$rc"; fatal $rc kt_compat ;;
    real_pmc)
      RE=${REAL_ENVS:-512}
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_real_$c" -o run -- python3 tools/bench_real_env.py --envs $RE --steps 3 --cpu 0 > "$OUT/pmc_real_$c.log" 2>&1
        rc=$?; echo "pmc real $c rc=$rc"; fatal $rc pmc_real_$c
      done
      python3 tools/pmc_real_summary.py "$OUT/pmc_real_FETCH_SIZE" "$OUT/pmc_real_WRITE_SIZE" "$OUT/pmc_real_step.json" --E $RE
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_real" -o run -- python3 tools/bench_real_env.py --envs $RE --steps 20 --cpu 0 > "$OUT/kt_real.log" 2>&1
      rc=$?; echo "kt real rc=$rc"; fatal $rc kt_real ;;
    real_sq)
      RE=${REAL_ENVS:-512}
      SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
      SQ2="SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_COUNT"
      i=1
      for set in "$SQ1" "$SQ2"; do
        timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/sq_real$i" -o run -- python3 tools/bench_real_env.py --envs $RE --steps 3 --cpu 0 > "$OUT/sq_real$i.log" 2>&1
        rc=$?; echo "sq real $i rc=$rc"; fatal $rc sq_real$i; i=$((i+1))
      done ;;
    *) echo "unknown step $st" ;;
  esac
done
exit 0
