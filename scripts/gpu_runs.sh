#!/bin/bash
# Parameterised bench runs on one GPU box (A/B pairs, window sweeps, shard checks): every run is
# one `python bench.py` line under its own time limit, alternated over REPS, into
# gpurun_out/$TAG/<name>_<rep>.json (+ .err).  The command line of each run is logged beside it
# (<name>_<rep>.cmd), so a cited record names the exact command that produced it.
#   RUNS="name|var|bench args;..."   var: "base" = the in-tree library, else
#                                    rs-pathplanning_amd/lib/<var>/libpathplanning_amd.so
#   REPS="1 2"                       repetitions (alternated: every run of rep 1, then rep 2, ...)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT="gpurun_out/${TAG:-runs}"
mkdir -p "$OUT"
IFS=';' read -ra JOBS <<< "$RUNS"
for rep in ${REPS:-1}; do
  for j in "${JOBS[@]}"; do
    IFS='|' read -r name var args <<< "$j"
    f="$OUT/${name}_${var}_$rep"
    lib="$R/rs-pathplanning_amd/lib/libpathplanning_amd.so"
    [ "$var" = base ] || lib="$R/rs-pathplanning_amd/lib/$var/libpathplanning_amd.so"
    # the library's hash before the run, so a run that fails before its line still names its build
    echo "lib_sha256_16 $(sha256sum "$lib" | cut -c1-16)" > "$f.lib"
    if [ "$var" = base ]; then
      echo "python -u bench.py $args" > "$f.cmd"
      timeout -k 10 ${LIMIT:-400} python -u bench.py $args > "$f.json" 2> "$f.err" || { echo "FAILED $name"; tail -20 "$f.err"; exit 1; }
    else
      echo "PP_AMD_LIB=rs-pathplanning_amd/lib/$var/libpathplanning_amd.so python -u bench.py $args --allow-variant-lib" > "$f.cmd"
      PP_AMD_LIB="$R/rs-pathplanning_amd/lib/$var/libpathplanning_amd.so" timeout -k 10 ${LIMIT:-400} python -u bench.py $args --allow-variant-lib > "$f.json" 2> "$f.err" || { echo "FAILED $name"; tail -20 "$f.err"; exit 1; }
    fi
    echo "ok $name $rep"
  done
done
