# query-batch active-task compaction: the -m gpu suite, then A/B against lib/head (the commit before)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05al4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=r05al4 REPS="1 2" WLS="config3" VARIANTS="base head" bash scripts/gpu_ab.sh || exit 1
TAG=r05al4 REPS="1 2" WLS="config3" VARIANTS="base head" EXTRA="--queries 1024" SFX=_shard bash scripts/gpu_ab.sh
