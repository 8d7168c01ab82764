# round 6: the walk's per-workgroup timeline with per-task point histogram (diagnostic build,
# scripts/diag_walk_timeline.py) for the shard, the full batch and its batch plan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06k
for wl in "c3s|--queries 1024" "c3|"; do
  IFS='|' read -r n a <<< "$wl"
  rm -f gpurun_out/r06k/$n.bin
  PP_DIAG_OUT=gpurun_out/r06k/$n.bin PP_AMD_LIB=rs-pathplanning_amd/lib/walktl/libpathplanning_amd.so timeout -k 10 300 python3 bench.py --workload config3 $a --no-cpu-baseline --allow-variant-lib > gpurun_out/r06k/$n.json 2> gpurun_out/r06k/$n.err || { tail -5 gpurun_out/r06k/$n.err; exit 1; }
  python3 scripts/diag_walk_timeline.py report gpurun_out/r06k/$n.bin > gpurun_out/r06k/$n.txt
  rm -f gpurun_out/r06k/$n.bin
  echo "tl $n ok"
done
