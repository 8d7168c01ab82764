# the batch walk's occupancy after the active-task list and K = 32: 5 waves for the shard (big32k),
# 5 waves everywhere (w5: no spill)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r05wv REPS="1 2" WLS="config3" VARIANTS="base w5" bash scripts/gpu_ab.sh || exit 1
TAG=r05wv REPS="1 2" WLS="config3" VARIANTS="base big32k" EXTRA="--queries 1024" SFX=_shard bash scripts/gpu_ab.sh
