#!/bin/bash
# Build a variant of libsemtsdf.so with extra compile definitions, for same-box A/B runs
# (SEMTSDF_LIB=build/var_NAME.so).  Usage: bash tools/build_variant.sh NAME [-DFOO=1 ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
mkdir -p $R/build
cd $R && python3 -c "import sys, __graft_entry__ as g; g.build_lib(force=True, extra_flags=sys.argv[2:], out=sys.argv[1])" \
  $R/build/var_$N.so "$@"
echo built build/var_$N.so
