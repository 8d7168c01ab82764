# round 6: analytic arc classes (variant lib/arc, built out of tree) — the parity, full-size,
# batch-plan and RRT* files on the variant (with the arc tangent test), then A/B against the
# in-tree library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06w
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k arc_shortcut -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06w/pytest_base_arc.log 2>&1 || { tail -30 gpurun_out/r06w/pytest_base_arc.log; exit 1; }
tail -1 gpurun_out/r06w/pytest_base_arc.log
PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/arc/libpathplanning_amd.so timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch_plan.py tests/test_gpu_rrtstar.py tests/test_gpu_polygons.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06w/pytest_arc.log 2>&1 || { tail -30 gpurun_out/r06w/pytest_arc.log; exit 1; }
tail -2 gpurun_out/r06w/pytest_arc.log
TAG=r06w REPS="1 2" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|arc|--workload config3 --queries 1024 --no-cpu-baseline;c3|base|--workload config3 --no-cpu-baseline;c3|arc|--workload config3 --no-cpu-baseline;c5|base|--workload config5 --no-cpu-baseline;c5|arc|--workload config5 --no-cpu-baseline;ex|base|--workload example_rrt --no-cpu-baseline;ex|arc|--workload example_rrt --no-cpu-baseline;pl|base|--workload plan --no-cpu-baseline;pl|arc|--workload plan --no-cpu-baseline" bash scripts/gpu_runs.sh
