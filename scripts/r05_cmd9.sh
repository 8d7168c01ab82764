# polygon S classes: the -m gpu suite, then example_rrt / plan / polygons A/B against the build
# without them (lib/nopolys), alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05ps
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=r05ps REPS="1 2" WLS="example_rrt plan" VARIANTS="base nopolys" bash scripts/gpu_ab.sh
