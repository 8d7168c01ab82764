#!/bin/bash
# config 5 (RRT*) per library variant, then a kernel trace of the config-3 plan; gpurun_out/$TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-c5ab}"
mkdir -p "$OUT"
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then
    timeout -k 10 300 python -u bench.py --workload config5 --no-cpu-baseline > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err" || { tail -20 "$OUT/c5_$v.err"; exit 1; }
  else
    PP_AMD_LIB="$PWD/rs-pathplanning_amd/lib/$v/libpathplanning_amd.so" timeout -k 10 300 python -u bench.py --workload config5 --no-cpu-baseline --allow-variant-lib > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err" || { tail -20 "$OUT/c5_$v.err"; exit 1; }
  fi
  echo "done c5 $v"
done
