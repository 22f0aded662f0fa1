#!/bin/bash
# PMC passes over a short bench run (integrate only).  Usage: bash tools/pmc_integrate.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--no-cpu-baseline --no-pipeline --steps 5 --warmup 1 --frames 4"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC" "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($ctr) rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
