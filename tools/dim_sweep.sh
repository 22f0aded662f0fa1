#!/bin/bash
# Integrate kernel time against the size of the frame's work: the C3 stream at several cubic
# volume sizes (fit t = a + b * live units: a is the per-launch fixed cost).
# Usage: bash tools/dim_sweep.sh "256 384 512 640 768"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in $1; do
  echo -n "dim $d: "
  timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-pipeline --steps 20 --dim $d 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('kernel_ms', d['integrate_kernel_ms'], 'prep_ms', d['prep_ms'], 'step_ms', d['ms_per_step'], 'live', d['live_units_per_frame'], 'free', d['free_units_per_frame'], 'touched', d['touched_per_frame'], 'gated', d['gated_per_frame'])" || exit 1
done
