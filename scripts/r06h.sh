set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r06h REPS="1 2" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|nsub1|--workload config3 --queries 1024 --no-cpu-baseline;c3s|wg3|--workload config3 --queries 1024 --no-cpu-baseline" bash scripts/gpu_runs.sh
