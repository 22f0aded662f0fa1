#!/bin/bash
# C2 (256^3 TSDF + i32 colour, ungated) diagnosis: the C2 record alone, PMC bytes and the
# instruction mix of its integrate kernel.  Usage: bash tools/diag_c2.sh TAG
set -u
TAG=${1:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "[c2] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
cd $R
timeout -k 10 300 python3 bench.py --only c2 --steps 20 > $O/c2.json 2> $O/c2.err
step bench $?
BENCH_ARGS="--only c2 --steps 10 --warmup 2" bash $R/tools/pmc_integrate.sh gpurun_out/$TAG/pmc FETCH_SIZE WRITE_SIZE \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" > $O/pmc.log 2>&1
step pmc $?
KER="k_integrate<false, false, false, false, false, false, true>"
python3 $R/tools/pmc_summary.py $O/pmc "$KER" > $O/pmc_summary.txt 2>&1
step pmc_summary $?
python3 $R/tools/traffic.py $O/pmc "$KER" $O/traffic.json 256 > $O/traffic.log 2>&1
step traffic $?
