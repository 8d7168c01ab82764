# round 6: the walk's record prefetch (variant lib/pf) against the in-tree library: the GPU parity
# files on the variant, then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06m2
PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/pf/libpathplanning_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06m2/pytest_pf.log 2>&1 || { tail -30 gpurun_out/r06m2/pytest_pf.log; exit 1; }
tail -2 gpurun_out/r06m2/pytest_pf.log
TAG=r06m2 REPS="1 2" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|pf|--workload config3 --queries 1024 --no-cpu-baseline;c3|base|--workload config3 --no-cpu-baseline;c3|pf|--workload config3 --no-cpu-baseline;c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2|pf|--workload config2 --no-cpu-baseline --no-size-sweep;c5|base|--workload config5 --no-cpu-baseline;c5|pf|--workload config5 --no-cpu-baseline" bash scripts/gpu_runs.sh
