#!/bin/bash
# VALU/SALU/VMEM instruction counts of k_integrate per timing probe (SEMTSDF_DEBUG_INTEGRATE)
set -u
for d in ${1:-0 3 4}; do
  SEMTSDF_DEBUG_INTEGRATE=$d bash tools/pmc_groups.sh gpurun_out/pmcd/d$d "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" > /dev/null || exit 1
  echo "== debug $d"; python3 tools/pmc_summary.py gpurun_out/pmcd/d$d "${KER:-k_integrate<true, true, false, false, false, false, true>}"
done
