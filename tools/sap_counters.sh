#!/bin/bash
# SAP selector issue counters (which unit binds the augmenting-path step): the counter list,
# then SQ passes over bench.py --selector sap for the in-tree library and each variant given.
#   bash tools/sap_counters.sh OUT_DIR [lib.so ...]
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --selector sap --cpu-baseline 0 --secondary 0 --steps 10 --warmup 3"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "counter list failed"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE"
# keep the counters this device lists (an unknown name fails the whole pass)
avail() { local out=""; for c in $1; do grep -qw "$c" "$OUT/counters.txt" && out="$out $c"; done; echo $out; }
P1=$(avail "$P1"); P2=$(avail "$P2")
echo "pass 1: $P1"; echo "pass 2: $P2"
for lib in default "$@"; do
  if [ "$lib" = default ]; then unset ASG_LIB_PATH; else export ASG_LIB_PATH=$PWD/$lib; fi
  tag=$(basename "$lib" .so)
  i=0
  for P in "$P1" "$P2"; do
    i=$((i + 1))
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/${tag}_p$i" -o run -- python3 $B \
        > "$OUT/${tag}_p$i.log" 2>&1 || { echo "FAILED $tag p$i"; tail -5 "$OUT/${tag}_p$i.log"; exit 1; }
    echo "ok $tag p$i"
  done
done
