set -o pipefail
mkdir -p gpurun_out/ab5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
for v in default build/nt1w3.so build/nt1w3x1.so build/nt1w4.so; do
  if [ $v = default ]; then timeout -k 5 120 python tools/agent_ab.py >> gpurun_out/ab5/ab.log 2>&1 || exit 1
  else ASG_LIB_PATH=$v timeout -k 5 120 python tools/agent_ab.py >> gpurun_out/ab5/ab.log 2>&1 || exit 1; fi
done; done
