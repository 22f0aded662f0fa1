# r04: PMC counters of the fused march, the decide and the map passes in the C3 pipeline
# (bench --only pipeline); one counter group per rocprofv3 pass.
set -u
O=gpurun_out/r04_ab32
mkdir -p $O
BENCH_ARGS="--only pipeline" bash tools/pmc_integrate.sh gpurun_out/r04_ab32/pmc \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" FETCH_SIZE > $O/pmc.log 2>&1
echo "pmc rc=$?" >> $O/steps.log
for k in "k_march_fused" "k_assoc_decide" "k_brick_oct_axis" "k_integrate<true, true, false, false, false, false, false>"; do
  echo "== $k" >> $O/pmc_summary.txt
  python3 tools/pmc_summary.py $O/pmc "$k" >> $O/pmc_summary.txt 2>&1
done
echo "summary rc=$?" >> $O/steps.log
