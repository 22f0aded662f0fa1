#!/bin/bash
# Integrate diagnosis on the GPU box (outputs under gpurun_out/TAG): the unit-order memory
# microbenchmark, the C3 integrate line, and two SQ counter passes of the integrate kernel
# (issue / wait split, SALU).  Usage: bash tools/diag_integrate.sh TAG
set -u
TAG=${1:-diag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "[diag] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
if [ -x $R/tools/membench_units ]; then
  timeout -k 10 120 $R/tools/membench_units > $O/membench_units.txt 2>&1
  step membench $?
fi
cd $R
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pipeline --steps 40 > $O/bench_c3.json 2> $O/bench_c3.err
step bench $?
BENCH_ARGS="--no-cpu-baseline --no-pipeline --steps 10 --warmup 2 --frames 4" bash $R/tools/pmc_integrate.sh gpurun_out/$TAG/pmc \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" > $O/pmc.log 2>&1
step pmc $?
python3 $R/tools/pmc_summary.py $O/pmc "k_integrate<true, true, false, false, false, false, true>" > $O/pmc_summary.txt 2>&1
step pmc_summary $?
