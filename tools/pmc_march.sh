#!/bin/bash
# PMC passes of the association march and the render raycast (pipeline section of the bench),
# one rocprofv3 run per counter group; per-dispatch means via tools/pmc_summary.py.
# Usage: bash tools/pmc_march.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$1
BENCH_ARGS="--only pipeline" bash $R/tools/pmc_groups.sh $OUT \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS" \
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH" \
  "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum" \
  "FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" > $R/$OUT.log 2>&1 || exit $?
for k in "k_render<false, true>" "k_assoc_march<true>"; do echo "== $k"; python3 $R/tools/pmc_summary.py $R/$OUT "$k"; done
