#!/bin/bash
# rocprofv3 kernel-trace stats of one bench run (pipeline included)
set -u
T=${1:-st}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/stats -o run -- python3 $R/bench.py --no-cpu-baseline ${BENCH_EXTRA:-} > $R/gpurun_out/$T/bench.json 2> $R/gpurun_out/$T/bench.err || exit $?
f=$(find $R/gpurun_out/$T/stats -name "run_kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:16]: print('%-70s %6s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
"
