# round 6: counter passes at the final library, part 2 (the window pipelines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r06pmcF2 WLS="config2 config4" bash scripts/gpu_pmc.sh
