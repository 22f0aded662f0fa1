#!/bin/bash
# Stall/issue counters of the integrate kernel, one rocprofv3 pass per group; a pass whose
# counter names the tool rejects is skipped, a time-out ends the script.
# Usage: bash tools/pmc_detail.sh OUTDIR [bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/pmcd}
shift
ARGS=${*:-"--no-cpu-baseline --no-pipeline --steps 10 --warmup 2"}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TCP_TCC_WRITE_REQ_sum TCC_EA0_WRREQ_STALL_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($ctr) rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
