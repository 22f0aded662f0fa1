#!/bin/bash
# Final measurement, part A: PMC traffic + counters of C3 and C2 (stamped with the build key)
set -u
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
KER="k_integrate<true, true, false, false, false, false, true>"
step() { echo "[measure] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
BENCH_ARGS="--no-cpu-baseline --no-pipeline --no-c4 --steps 10 --warmup 2 --frames 4" bash $R/tools/pmc_integrate.sh gpurun_out/$TAG/pmc \
  FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" > $O/pmc.log 2>&1
step pmc $?
python3 $R/tools/traffic.py $O/pmc "$KER" $O/traffic.json 512 > $O/traffic.log 2>&1
step traffic $?
python3 $R/tools/pmc_summary.py $O/pmc "$KER" > $O/pmc_summary.txt 2>&1
step pmc_summary $?
bash $R/tools/diag_c2.sh $TAG/c2 > $O/c2.log 2>&1
step c2 $?
