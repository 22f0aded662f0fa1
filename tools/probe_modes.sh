#!/bin/bash
# Integrate timing probes (build/var_probes.so, -DSEMTSDF_INTEGRATE_PROBES=1) per SEMTSDF_DEBUG_INTEGRATE mode:
# 0 normal, 3 no state traffic, 21 no state traffic + one-address gathers, 4 no colour/histogram
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for m in "$@"; do
  echo -n "[mode $m] "
  SEMTSDF_LIB=$R/build/var_probes.so SEMTSDF_DEBUG_INTEGRATE=$m timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-pipeline --steps 30 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', d['integrate_kernel_ms'], 'step_ms', d['ms_per_step'])" || exit 1
done
