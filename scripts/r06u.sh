# round 6: nn_finalize's near-tie rescan of the appended nodes from each lane's top-2 (variant
# lib/nnfin, built out of tree) — parity files on the variant, then A/B on configs 2 and 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06u
PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/nnfin/libpathplanning_amd.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_libm_flips.py tests/test_gpu_polygons.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06u/pytest_nnfin.log 2>&1 || { tail -30 gpurun_out/r06u/pytest_nnfin.log; exit 1; }
tail -2 gpurun_out/r06u/pytest_nnfin.log
TAG=r06u REPS="1 2 3" RUNS="c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2|nnfin|--workload config2 --no-cpu-baseline --no-size-sweep;c4|base|--workload config4 --no-cpu-baseline --no-size-sweep;c4|nnfin|--workload config4 --no-cpu-baseline --no-size-sweep" bash scripts/gpu_runs.sh
