#!/bin/bash
# Kernel + copy trace of the C3 pipeline section (bench --only pipeline) for timeline analysis
# (tools/timeline.py).  Usage: bash tools/trace_pipeline.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --only pipeline > $O/bench.json 2> $O/bench.err
