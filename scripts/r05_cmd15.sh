# first chunk's pd loads hoisted before the record reads: A/B against lib/nopre, then the suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r05pre REPS="1 2" WLS="config2 config4 config3" VARIANTS="base nopre" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh || exit 1
TAG=r05pre REPS="1 2" WLS="config3" VARIANTS="base nopre" EXTRA="--queries 1024" SFX=_shard bash scripts/gpu_ab.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r05pre/pytest.log 2>&1 || { tail -40 gpurun_out/r05pre/pytest.log; exit 1; }
tail -2 gpurun_out/r05pre/pytest.log
