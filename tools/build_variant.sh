#!/bin/bash
# Build a variant of libsemtsdf.so with extra compile definitions, for same-box A/B runs
# (SEMTSDF_LIB=build/var_NAME.so).  Usage: bash tools/build_variant.sh NAME [-DFOO=1 ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
mkdir -p $R/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 "$@" \
  $R/slam-maskrcnn_amd/csrc/semtsdf_kernels.hip $R/slam-maskrcnn_amd/csrc/semtsdf_api.cpp -o $R/build/var_$N.so
echo built build/var_$N.so
