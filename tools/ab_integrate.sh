#!/bin/bash
# Same-box A/B of library builds on the C3 integrate line (no CPU baseline, no pipeline):
# bash tools/ab_integrate.sh LIB1.so LIB2.so ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$@"; do
  echo -n "[$lib] "
  SEMTSDF_LIB=$R/$lib timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-pipeline --steps 40 ${AB_ARGS:-} 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('kernel_ms', d['integrate_kernel_ms'], 'prep_ms', d['prep_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'live', d['live_units_per_frame'], 'free', d['free_units_per_frame'], 'full', d.get('full_free_units_per_frame'), 'touched', d['touched_per_frame'], 'gated', d['gated_per_frame'], 'lazy', d.get('lazy_weight_voxels_per_frame'))" || exit 1
done
