# the batch NN's node loop unrolled 8 / 16 (more row loads in flight) against 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r05un REPS="1 2" WLS="config3" VARIANTS="base u8 u16" bash scripts/gpu_ab.sh || exit 1
TAG=r05un REPS="1 2" WLS="config3" VARIANTS="base u8 u16" EXTRA="--queries 1024" SFX=_shard bash scripts/gpu_ab.sh
