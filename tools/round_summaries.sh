#!/bin/bash
# Summaries of a tools/round_profile.sh run into profiles/ (CPU, after the gpurun call):
#   bash tools/round_summaries.sh gpurun_out/round_sN TAG [ROUND=r4]   (files profiles/ROUND_*_TAG.*)
# per-tile figures count the 20 selection passes of one whole-episode launch (--rows E n 20)
set -e
R=${1:?round dir}; T=${2:?tag}; RN=${3:-r4}
P=profiles
for v in "rnn::64:64:16384:1" "lin:_lin:64:64:16384:0" "c4:_256:256:256:2048:1"; do
  IFS=: read tag sfx n m E rnn <<< "$v"
  w="--n $n --m $m --L 3 --E $E --steps-per-launch 20 --use-rnn $rnn"
  python tools/pmc_summary.py $R/fetch_$tag $R/write_$tag $P/${RN}_pmc_rollout_kernel${sfx}_$T.json --kernel rollout_kernel --fetch-doubled $w
  python tools/pmc_agent_summary.py $R/sq1_$tag $R/kt_$tag/run_kernel_stats.csv $P/${RN}_pmc_rollout_sq${sfx}_$T.json --kernel rollout_kernel --rows $((E * n * 20)) $w
  python tools/pmc_agent_summary.py $R/sq2_$tag $R/kt_$tag/run_kernel_stats.csv $P/${RN}_pmc_rollout_issue2${sfx}_$T.json --kernel rollout_kernel --rows $((E * n * 20)) $w
  cp $R/kt_$tag/run_kernel_stats.csv $P/${RN}_kernel_stats_${tag}_$T.csv
done
w="--n 64 --m 64 --L 3 --E 16384 --steps-per-launch 1 --use-rnn 0"
if [ -d $R/fetch_q ]; then
  python tools/pmc_summary.py $R/fetch_q $R/write_q $P/${RN}_pmc_rollout_q_kernel_$T.json --kernel rollout_kernel --fetch-doubled $w
  python tools/pmc_agent_summary.py $R/sq1_q $R/kt_sap/run_kernel_stats.csv $P/${RN}_pmc_rollout_q_sq_$T.json --kernel rollout_kernel --rows $((16384 * 64)) $w
fi
cp $R/kt_sap/run_kernel_stats.csv $P/${RN}_kernel_stats_sap_$T.csv
python tools/pmc_sap_summary.py $R/sq_sap $R/bench_sap.log $P/${RN}_pmc_sap_kernel_$T.json
if [ -d $R/fetch_c1 ]; then
  python tools/pmc_summary.py $R/fetch_c1 $R/write_c1 $P/${RN}_pmc_random_rollout_$T.json --kernel random_rollout_kernel \
      --n 16 --m 16 --L 3 --E 4096 --steps-per-launch 20 --use-rnn 0 --fetch-doubled
  cp $R/kt_c1/run_kernel_stats.csv $P/${RN}_kernel_stats_c1_$T.csv
fi
