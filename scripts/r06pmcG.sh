# round 6, final: the counter passes of every workload at the record's library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r06pmcG WLS="${WLS:-config3 config3s config5 config2 config4}" bash scripts/gpu_pmc.sh
