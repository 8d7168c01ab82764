#!/bin/bash
# A/B of library variants (rs-pathplanning_amd/lib/<variant>/) against the in-tree build on one
# box: for each workload in WLS, every variant in VARIANTS (base = in-tree), bench lines into
# gpurun_out/$TAG/<wl>_<variant>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-ab}"
mkdir -p "$OUT"
for rep in ${REPS:-1}; do
for wl in ${WLS:-config3}; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then
      timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline $EXTRA > "$OUT/${wl}_${v}_${rep}${SFX}.json" 2> "$OUT/${wl}_${v}_${rep}${SFX}.err" || { tail -20 "$OUT/${wl}_${v}_${rep}${SFX}.err"; exit 1; }
    else
      PP_AMD_LIB="$PWD/rs-pathplanning_amd/lib/$v/libpathplanning_amd.so" timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --allow-variant-lib $EXTRA > "$OUT/${wl}_${v}_${rep}${SFX}.json" 2> "$OUT/${wl}_${v}_${rep}${SFX}.err" || { tail -20 "$OUT/${wl}_${v}_${rep}${SFX}.err"; exit 1; }
    fi
    echo "done $wl $v $rep"
  done
done
done
