# round 6: the walk's per-workgroup timeline (diagnostic build, scripts/diag_walk_timeline.py) for
# the shard and the full batch, the config-3 batch plan's dispatch timeline (steer rounds), then the
# config-3 / config-2 counter passes at the record library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06j/tl
for wl in "c3s|--queries 1024" "c3|"; do
  IFS='|' read -r n a <<< "$wl"
  rm -f gpurun_out/r06j/tl/$n.bin
  PP_DIAG_OUT=gpurun_out/r06j/tl/$n.bin PP_AMD_LIB=rs-pathplanning_amd/lib/walktl/libpathplanning_amd.so timeout -k 10 300 python3 bench.py --workload config3 $a --no-cpu-baseline --allow-variant-lib > gpurun_out/r06j/tl/$n.json 2> gpurun_out/r06j/tl/$n.err || { tail -5 gpurun_out/r06j/tl/$n.err; exit 1; }
  python3 scripts/diag_walk_timeline.py report gpurun_out/r06j/tl/$n.bin > gpurun_out/r06j/tl/$n.txt
  rm -f gpurun_out/r06j/tl/$n.bin
  echo "tl $n ok"
done
TAG=r06j RUNS="c3|base|--workload config3 --no-cpu-baseline" bash scripts/gpu_trace_var.sh
python3 scripts/plan_timeline.py gpurun_out/r06j/c3 > gpurun_out/r06j/c3_plan_timeline.json
find gpurun_out/r06j -name "*kernel_trace.csv" -delete
TAG=r06pmc WLS="config3 config2" bash scripts/gpu_pmc.sh
