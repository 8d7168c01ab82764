#!/bin/bash
# Round-4 check: the -m gpu tests, then config 3 (full batch and the 1024-query shard) per library
# variant (VARIANTS; base = in-tree), the batch plan on one kernel (PP_AMD_CF_ROUNDS=0) and a
# config-2 line; everything under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-cfr}"
mkdir -p "$OUT"
if [ "${TESTS:-all}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -3 "$OUT/pytest.log"
fi
run() {  # name, lib variant, bench args
  local name=$1 v=$2; shift 2
  if [ "$v" = base ]; then
    timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  else
    PP_AMD_LIB="$PWD/rs-pathplanning_amd/lib/$v/libpathplanning_amd.so" timeout -k 10 300 python -u bench.py --no-cpu-baseline --allow-variant-lib "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  fi
  echo "done $name"
}
for v in ${VARIANTS:-base}; do
  run "c3_$v" "$v" --workload config3
  run "c3s_$v" "$v" --workload config3 --queries 1024
done
PP_AMD_CF_ROUNDS=0 run c3_base_onekernel base --workload config3
run c2_base base --warmup 3 --no-sub
