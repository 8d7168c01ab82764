# round 6: the batch NN on two waves per query (variant lib/nnsplit, built out of tree from the
# parked patch) — parity files on the variant, then A/B against the in-tree library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06r
PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/nnsplit/libpathplanning_amd.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch_plan.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06r/pytest_nnsplit.log 2>&1 || { tail -30 gpurun_out/r06r/pytest_nnsplit.log; exit 1; }
tail -2 gpurun_out/r06r/pytest_nnsplit.log
TAG=r06r REPS="1 2 3" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|nnsplit|--workload config3 --queries 1024 --no-cpu-baseline;c3|base|--workload config3 --no-cpu-baseline;c3|nnsplit|--workload config3 --no-cpu-baseline" bash scripts/gpu_runs.sh
