#!/bin/bash
# Build libsemtsdf.so from the library sources of git revision REV (same hipcc flags as
# __graft_entry__.build_lib), for same-box A/B runs against the working tree's build
# (SEMTSDF_LIB=build/rev_NAME.so).  Usage: bash tools/build_commit.sh REV NAME [-DFOO=1 ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; N=$2; shift 2
T=$(mktemp -d)
cd $R && git archive $REV slam-maskrcnn_amd/csrc include | tar -x -C $T
mkdir -p $R/build
python3 - "$T" "$R/build/rev_$N.so" "$@" <<'PY'
import subprocess, sys
sys.path.insert(0, ".")
import __graft_entry__ as g
t, out, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
srcs = [f"{t}/slam-maskrcnn_amd/csrc/semtsdf_kernels.hip", f"{t}/slam-maskrcnn_amd/csrc/semtsdf_api.cpp"]
subprocess.check_call(["/opt/rocm/bin/hipcc", *g.HIPCC_FLAGS, *extra, f"-I{t}/include", '-DSEMTSDF_BUILD_KEY="rev"', *srcs, "-o", out])
PY
rm -rf $T
echo built build/rev_$N.so
