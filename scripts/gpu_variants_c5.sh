#!/bin/bash
# Config 5 bench lines for library variants (lib/v_<name>), alternated: VARIANTS="base a b".
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/var5${TAGS:-}"
mkdir -p "$OUT"
cd "$R"
for rep in 1 2; do
  for v in ${VARIANTS:-base}; do
    PP_AMD_LIB="$R/rs-pathplanning_amd/lib/v_$v/libpathplanning_amd.so" timeout -k 10 300 python3 bench.py --workload ${WL:-config5} --no-cpu-baseline --allow-variant-lib ${BENCH_ARGS:-} > "$OUT/b_${v}_$rep.json" 2> "$OUT/b_${v}_$rep.err" || { tail -20 "$OUT/b_${v}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$rep.json')); print('$v', round(d['value']/1e6,2), 'M it/s', d.get('records_digest'), d.get('best_length'), d.get('check_finish_ms'))"
  done
done
echo var5-done
