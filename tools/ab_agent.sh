#!/bin/bash
# A/B of agent-kernel builds on one MI355X: tools/agent_ab.py per library, alternating,
# each in its own process.  Usage: tools/ab_agent.sh OUTDIR "label=lib[:ENV=VAL]" ...
#   lib "default" = the in-tree library
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 3; do
  for spec in "$@"; do
    label=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*:}
    if [ "$lib" = default ]; then libenv=""; else libenv="ASG_LIB_PATH=$lib"; fi
    echo -n "$label " >> "$OUT/ab.log"
    env $libenv $envs timeout -k 5 120 python tools/agent_ab.py >> "$OUT/ab.log" 2>&1 || exit 1
  done
done
