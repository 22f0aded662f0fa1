#!/bin/bash
# One measurement round on the GPU box: PMC traffic of the timed integrate kernel, the bench
# line (reads that traffic), a rocprofv3 kernel-trace --stats run of the same bench, and a
# 2-rank rehearsal of the sharded bench on one GPU (gloo control plane).
# Usage: bash tools/measure.sh TAG     (outputs under gpurun_out/TAG)
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
KER="k_integrate<true, true, false, false, false, false, true>"
step() { echo "[measure] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }

BENCH_ARGS="--no-cpu-baseline --no-pipeline" bash $R/tools/pmc_integrate.sh gpurun_out/$TAG/pmc FETCH_SIZE WRITE_SIZE > $O/pmc.log 2>&1
step pmc $?
python3 $R/tools/traffic.py $O/pmc "$KER" $O/traffic.json 512 > $O/traffic.log 2>&1
step traffic $?
cd $R
timeout -k 10 600 python3 bench.py --traffic-json $O/traffic.json > $O/bench.json 2> $O/bench.err
step bench $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --no-cpu-baseline --traffic-json $O/traffic.json > $O/bench_prof.json 2> $O/bench_prof.err
step rocprof_stats $?
cd $R
BENCH_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_n2.json 2> $O/bench_n2.err
step rehearsal_n2 $?
