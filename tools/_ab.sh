#!/bin/bash
# A/B of integrate variants on one box: bash tools/_ab.sh "ENV1=.. ENV2=.." "..."
# Each config runs ROUNDS times (default 2), interleaved, kernel timing only.
set -u
R=${ROUNDS:-2}
for r in $(seq $R); do
for e in "$@"; do
  echo -n "[$e] "
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pipeline --steps ${STEPS:-40} 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value'], 'kernel_ms', d['integrate_kernel_ms'], 'prep_ms', d['prep_ms'], 'step_ms', d['ms_per_step'], 'touched', d['touched_per_frame'], 'frac', d['roofline']['frac'])" || exit 1
done
done
