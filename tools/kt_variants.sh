#!/bin/bash
# kernel stats per library variant: bash kt_variants.sh OUT lib...
OUT=$1; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
for lib in "$@"; do
  n=$(basename $(dirname $lib))
  ASG_LIB_PATH=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 tools/bench_real_env.py --envs 512 --steps 20 --cpu 0 > $OUT/$n.log 2>&1 || { echo "fail $n"; exit 1; }
done
