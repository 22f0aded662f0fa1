#!/bin/bash
# Timing probes of the integrate kernel (SEMTSDF_DEBUG_INTEGRATE): 0 normal, 3 classify only,
# 4 no gated traffic, 6 no histogram atomics, 9 no depth gather, 10 no sdf/weight stores,
# 1xx fraction xx/8 of the resident grid.  Usage: bash tools/probe_sweep.sh "0 3 4 ..."
set -u
for d in ${1:-"0 3 4 6 9 10"}; do
  echo -n "debug $d: "
  SEMTSDF_DEBUG_INTEGRATE=$d bash tools/probe_integrate.sh || exit $?
done
