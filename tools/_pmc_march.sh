#!/bin/bash
set -u
BENCH_ARGS="--no-cpu-baseline --steps 16 --warmup 2 --frames 16" bash tools/pmc_groups.sh gpurun_out/pmcm "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum" > /dev/null || exit 1
for k in k_render k_assoc_march; do echo "== $k"; python3 tools/pmc_summary.py gpurun_out/pmcm "$k"; done
