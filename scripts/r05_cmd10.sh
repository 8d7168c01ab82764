# check_finish phase timing (cftime variant) against the in-tree counts, transit and bench6_open
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05cft
mkdir -p $OUT
for sc in transit bench6_open; do
  timeout -k 10 120 python -u scripts/diag_cf_phases.py $sc > $OUT/base_$sc.json 2> $OUT/base_$sc.err || { tail -20 $OUT/base_$sc.err; exit 1; }
  PP_AMD_LIB="$PWD/rs-pathplanning_amd/lib/cftime/libpathplanning_amd.so" timeout -k 10 120 python -u scripts/diag_cf_phases.py $sc > $OUT/cftime_$sc.json 2> $OUT/cftime_$sc.err || { tail -20 $OUT/cftime_$sc.err; exit 1; }
done
cat $OUT/*.json
