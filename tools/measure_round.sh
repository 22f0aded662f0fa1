#!/bin/bash
# One measurement round on the GPU box (outputs under gpurun_out/TAG):
#   pmc/       FETCH_SIZE, WRITE_SIZE and instruction/occupancy/wait counters of the bench's integrate
#   traffic.json       per-launch HBM bytes of the timed C3 integrate kernel, stamped with the build key
#   c2/traffic.json    the same for the C2 kernel
#   bench.json     the bench line (CPU baseline included) reading both traffic records
#   stats/         rocprofv3 --kernel-trace --stats of the same bench (no CPU baseline)
#   pmcm/          march counters (association + render) over the pipeline section
# Usage: bash tools/measure_round.sh TAG
set -u
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
KER="k_integrate<true, true, false, false, false, false, true>"
step() { echo "[measure] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
BENCH_ARGS="--no-cpu-baseline --no-pipeline --steps 10 --warmup 2 --frames 4" bash $R/tools/pmc_integrate.sh gpurun_out/$TAG/pmc \
  FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" "TA_TA_BUSY_sum TD_TD_BUSY_sum TCC_HIT_sum TCC_MISS_sum" > $O/pmc.log 2>&1
step pmc $?
python3 $R/tools/traffic.py $O/pmc "$KER" $O/traffic.json 512 > $O/traffic.log 2>&1
step traffic $?
python3 $R/tools/pmc_summary.py $O/pmc "$KER" > $O/pmc_summary.txt 2>&1
step pmc_summary $?
bash $R/tools/diag_c2.sh $TAG/c2 > $O/c2.log 2>&1
step c2 $?
cd $R
timeout -k 10 600 python3 bench.py --traffic-json $O/traffic.json --c2-traffic-json $O/c2/traffic.json > $O/bench.json 2> $O/bench.err
step bench $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --no-cpu-baseline --no-pipeline --traffic-json $O/traffic.json > $O/bench_prof.json 2> $O/bench_prof.err
step rocprof_stats $?
cd $R
bash $R/tools/pmc_march.sh gpurun_out/$TAG/pmcm > $O/pmcm_summary.txt 2>&1
step pmc_march $?
