# S chord untested (chunk cut before it): the -m gpu suite, then A/B against lib/nochord
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05ch
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=r05ch REPS="1 2" WLS="example_rrt plan config3 config5" VARIANTS="base nochord" bash scripts/gpu_ab.sh
TAG=r05ch REPS="1 2" WLS="config3" VARIANTS="base nochord" EXTRA="--queries 1024" SFX=_shard bash scripts/gpu_ab.sh
