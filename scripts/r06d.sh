set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06d
rm -f gpurun_out/fin_stamps.txt
TAG=r06d REPS="1" RUNS="c2|finst|--workload config2 --no-cpu-baseline --no-size-sweep;c3|base|--workload config3 --no-cpu-baseline" bash scripts/gpu_runs.sh
mv gpurun_out/fin_stamps.txt gpurun_out/r06d/fin_stamps.txt
