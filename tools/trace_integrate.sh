#!/bin/bash
# Per-wave phase trace of k_integrate on the C3 bench stream (build first, on the CPU:
#   bash tools/build_variant.sh wtrace -DSEMTSDF_WAVE_TRACE=1 [other -D...]).
# Usage on the GPU box: bash tools/trace_integrate.sh OUTDIR [VARIANT]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/wtrace}
V=${2:-wtrace}
mkdir -p $O
rm -f $O/trace_$V.bin
SEMTSDF_LIB=$R/build/var_$V.so SEMTSDF_WAVE_TRACE=$O/trace_$V.bin timeout -k 10 300 \
  python3 $R/bench.py --no-cpu-baseline --no-pipeline --steps 10 --warmup 2 > $O/bench_$V.json 2> $O/bench_$V.err || exit $?
python3 $R/tools/wave_trace.py $O/trace_$V.bin ${ORDER:-free-first} > $O/summary_$V.txt 2>&1; rc=$?; rm -f $O/trace_$V.bin; exit $rc
