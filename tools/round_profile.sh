#!/bin/bash
# Round evidence on one MI355X (run through gpurun from the repo root):
#   bash tools/round_profile.sh OUT_DIR
# The headline schedule (configs[2]: the whole-episode fused rollout kernel, asg_rollout):
# rocprofv3 kernel statistics of the default bench, then separate PMC passes -- FETCH_SIZE,
# WRITE_SIZE, two SQ sets -- over one 20-step (whole-episode) launch per run; the same for
# the Linear agent (--use-rnn 0, mock_constellation_iql.yaml's agent) and configs[4]
# (256 x 256 dense); kernel statistics of the SAP leg and its SQ pass.  Every GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --cpu-baseline 0 --secondary 0"
E1="--steps 20 --warmup 0"   # one launch = one whole episode (20 steps)
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
SQ2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
prof() {  # prof NAME TIMEOUT rocprof-args -- bench-args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to rocprofv3 "$@" > "$OUT/$name.log" 2>&1 || { echo "FAILED $name"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "ok $name"
}
for v in "rnn:--use-rnn 1:2" "lin:--use-rnn 0:2" "c4:--use-rnn 1:4"; do
  tag=${v%%:*}; rest=${v#*:}; args=${rest%:*}; cfg=${rest##*:}
  prof kt_$tag 400 --kernel-trace --stats --output-format csv -d "$OUT/kt_$tag" -o run -- python3 $B $args --config $cfg
  prof fetch_$tag 400 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$tag" -o run -- python3 $B $args --config $cfg $E1
  prof write_$tag 400 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$tag" -o run -- python3 $B $args --config $cfg $E1
  prof sq1_$tag 400 --pmc $SQ1 --output-format csv -d "$OUT/sq1_$tag" -o run -- python3 $B $args --config $cfg $E1
  prof sq2_$tag 400 --pmc $SQ2 --output-format csv -d "$OUT/sq2_$tag" -o run -- python3 $B $args --config $cfg $E1
done
# the REDA step schedule's rollout kernel (asg_step_forward, Q written; the Linear agent of
# mock_constellation_reda.yaml): one launch per step
for v in "q:--selector sap --use-rnn 0:2"; do
  tag=${v%%:*}; rest=${v#*:}; args=${rest%:*}; cfg=${rest##*:}
  prof fetch_$tag 400 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$tag" -o run -- python3 $B $args --config $cfg $E1
  prof write_$tag 400 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$tag" -o run -- python3 $B $args --config $cfg $E1
  prof sq1_$tag 400 --pmc $SQ1 --output-format csv -d "$OUT/sq1_$tag" -o run -- python3 $B $args --config $cfg $E1
done
# BASELINE configs[1]: the random policy's episode kernel (asg_random_rollout)
prof kt_c1 300 --kernel-trace --stats --output-format csv -d "$OUT/kt_c1" -o run -- python3 $B --config 1
prof fetch_c1 300 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_c1" -o run -- python3 $B --config 1 $E1
prof write_c1 300 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_c1" -o run -- python3 $B --config 1 $E1
prof kt_sap 400 --kernel-trace --stats --output-format csv -d "$OUT/kt_sap" -o run -- python3 $B --selector sap --steps 20 --warmup 5
timeout -k 10 300 python bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 20 --warmup 5 > "$OUT/bench_sap.log" 2>&1 || exit 1
prof sq_sap 400 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq_sap" -o run -- python3 $B --selector sap --steps 20 --warmup 5
echo done
