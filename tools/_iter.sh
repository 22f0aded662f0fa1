#!/bin/bash
# iteration check: GPU parity tests, A/B timings, VALU/SALU/LDS instruction counts of the block kernel
set -u
T=${1:-it}
mkdir -p gpurun_out/$T
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$T/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/$T/pytest.log | head -20; exit $rc; }
bash tools/_ab.sh SEMTSDF_DEBUG_INTEGRATE=0 SEMTSDF_DEBUG_INTEGRATE=3 SEMTSDF_DEBUG_INTEGRATE=4 || exit 1
bash tools/pmc_groups.sh gpurun_out/$T/pmc "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" > /dev/null || exit 1
python3 tools/pmc_summary.py gpurun_out/$T/pmc "k_integrate<true, true, false, false, false, false, true>"
