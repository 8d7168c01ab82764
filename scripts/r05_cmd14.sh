# line kernel's closed-form generator: -m gpu suite, A/B against lib/nocf (serial chain)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05ln2
mkdir -p $OUT
# (suite passed in r05ln) timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
true
TAG=r05ln2 REPS="1 2" WLS="plan example_rrt" VARIANTS="base nocf" bash scripts/gpu_ab.sh || exit 1
TAG=r05ln2 REPS="1" WLS="config3" VARIANTS="base nocf" EXTRA="--detail gpurun_out/r05ln2/d.json" bash scripts/gpu_ab.sh
