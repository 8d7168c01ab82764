#!/bin/bash
# Round 4: the persistent query-batch kernel — the batch parity tests, then config-3 bench lines
# (full batch and a 1024-query shard) for both schedules and the library variants in VARIANTS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-pq}"
mkdir -p "$OUT"
if [ "${TESTS:-batch}" != "none" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_polygons.py tests/test_gpu_api_surface.py -x -q -m gpu -k "${TESTS_K:-batch or none_tree}" --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -3 "$OUT/pytest.log"
fi
for q in ${QUERIES:-8192 1024}; do
  for sch in ${SCHEDULES:-persistent lockstep}; do
    for v in ${VARIANTS:-base}; do
      if [ "$v" = base ]; then LIBENV=""; ALLOW=""; else LIBENV="PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/$v/libpathplanning_amd.so"; ALLOW="--allow-variant-lib"; fi
      env $LIBENV timeout -k 10 300 python -u bench.py --workload config3 --queries $q --schedule $sch --no-cpu-baseline $ALLOW $EXTRA > "$OUT/c3_${q}_${sch}_${v}.json" 2> "$OUT/c3_${q}_${sch}_${v}.err" || { tail -20 "$OUT/c3_${q}_${sch}_${v}.err"; exit 1; }
      echo "done $q $sch $v"
    done
  done
done
