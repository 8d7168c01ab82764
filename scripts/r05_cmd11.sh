# check_finish differential: prep twice / walk twice per edge against the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05cfe
mkdir -p $OUT
for rep in 1 2; do
for v in base edge2; do
for sc in transit bench6_open; do
  if [ $v = base ]; then unset PP_AMD_LIB; else export PP_AMD_LIB="$PWD/rs-pathplanning_amd/lib/$v/libpathplanning_amd.so"; fi
  timeout -k 10 120 python -u scripts/diag_cf_phases.py $sc > $OUT/${v}_${sc}_$rep.json 2> $OUT/${v}_${sc}_$rep.err || { tail -20 $OUT/${v}_${sc}_$rep.err; exit 1; }
done; done; done
grep -h . $OUT/*.json
