#!/bin/bash
# Build library variants into rs-pathplanning_amd/lib/v_<name>/ from "name:flags" pairs.
R="$(cd "$(dirname "$0")/.." && pwd)"
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  mkdir -p "$R/rs-pathplanning_amd/lib/v_$name"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off $flags \
    -o "$R/rs-pathplanning_amd/lib/v_$name/libpathplanning_amd.so" \
    "$R/rs-pathplanning_amd/csrc/pp_kernels.hip" "$R/rs-pathplanning_amd/csrc/pp_capi.cpp" \
    "$R/rs-pathplanning_amd/csrc/pp_scene.cpp" &
done
wait
