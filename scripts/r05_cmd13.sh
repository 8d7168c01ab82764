# batch walk tuning after the chord change: 5 waves for the full batch (w5), S threshold 32 / 128
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r05tu REPS="1 2" WLS="config3" VARIANTS="base w5 s32 s128" bash scripts/gpu_ab.sh || exit 1
TAG=r05tu REPS="1 2" WLS="config3" VARIANTS="base s32 s128" EXTRA="--queries 1024" SFX=_shard bash scripts/gpu_ab.sh || exit 1
TAG=r05tu REPS="1" WLS="config5 example_rrt" VARIANTS="base s32 s128" bash scripts/gpu_ab.sh
