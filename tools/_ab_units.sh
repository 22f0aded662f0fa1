#!/bin/bash
# A/B of integrate variants reporting live units: bash tools/_ab_units.sh "ENV1=.." "..."
set -u
for r in $(seq ${ROUNDS:-2}); do
for e in "$@"; do
  echo -n "[$e] "
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pipeline --steps ${STEPS:-40} 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('kernel_ms', d['integrate_kernel_ms'], 'prep_ms', d['prep_ms'], 'step_ms', d['ms_per_step'], 'units', d['live_bricks_per_frame'], 'touched', d['touched_per_frame'])" || exit 1
done
done
