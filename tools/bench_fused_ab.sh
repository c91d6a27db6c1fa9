set -o pipefail
cd $GRAFT_REPO_ROOT
for f in 0 1 0 1; do timeout -k 10 300 python bench.py --cpu-baseline 0 --secondary 0 --fused-rollout $f || exit 1; done
