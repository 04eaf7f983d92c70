#!/bin/bash
# Build a diagnostic / A-B variant of libgpfit: scripts/build_variant.sh NAME [-DFLAG ...]
# -> gaussian-process_amd/libgpfit_NAME.so (same sources and flags as __graft_entry__.build()).
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-value \
  -Wno-unused-result -mllvm --amdgpu-mfma-vgpr-form "$@" gaussian-process_amd/csrc/gpfit_api.hip -o gaussian-process_amd/libgpfit_$name.so \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
