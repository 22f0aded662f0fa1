#!/bin/bash
# Final measurement, part B: the bench line reading part A's traffic records, rocprofv3
# kernel stats of the C3 bench, march counters
set -u
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "[measure] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
cd $R
timeout -k 10 600 python3 bench.py --traffic-json profiles/traffic_latest.json --c2-traffic-json profiles/traffic_c2_latest.json > $O/bench.json 2> $O/bench.err
step bench $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --no-cpu-baseline --no-pipeline --no-c4 --traffic-json $R/profiles/traffic_latest.json > $O/bench_prof.json 2> $O/bench_prof.err
step rocprof_stats $?
