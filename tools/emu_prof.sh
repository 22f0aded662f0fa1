#!/bin/bash
# rocprofv3 kernel trace of tools/emu_composite.py for a library build; per-step means of k_shard_ray_step
# Usage: bash tools/emu_prof.sh OUTNAME [LIB.so]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
LIB=${2:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$LIB" ]; then export SEMTSDF_LIB=$R/$LIB; fi
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/tools/emu_composite.py 8 5 > $O/emu.log 2>&1 || exit $?
python3 - "$O" <<'PY'
import csv, glob, sys
import numpy as np
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_shard_ray_step" in r["Kernel_Name"]]
d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]).reshape(-1, 3, 8)
print("k_shard_ray_step mean us per step:", d.mean(axis=(0, 2)).round(1), "per view (8 shards):", d.sum(axis=(1, 2)).mean().round(1))
PY
cat $O/emu.log | grep -v amdgpu.ids
