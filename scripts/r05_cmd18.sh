# window steer over the live samples only (wlist): the -m gpu suite, then A/B against lib/head
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05wl
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=r05wl REPS="1 2" WLS="config2 config4" VARIANTS="base head" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh || exit 1
TAG=r05wl REPS="1" WLS="config1 plan" VARIANTS="base head" bash scripts/gpu_ab.sh
