# three sub-batch streams (lib/ns3) against two, with the active-task list
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r05ns REPS="1 2" WLS="config3" VARIANTS="base ns3" bash scripts/gpu_ab.sh || exit 1
TAG=r05ns REPS="1 2" WLS="config3" VARIANTS="base ns3" EXTRA="--queries 1024" SFX=_shard bash scripts/gpu_ab.sh
