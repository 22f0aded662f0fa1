#!/bin/bash
# Pipeline fields of bench.py for library variants, interleaved: bash tools/_pipe_cmp.sh LIB1 LIB2 ...
set -u
for r in $(seq ${ROUNDS:-2}); do
for l in "$@"; do
  echo -n "[$l] "
  SEMTSDF_LIB=$l timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps ${STEPS:-30} 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']
print('kernel_ms', d['integrate_kernel_ms'], 'pipe_ms', round(p['ms_per_frame'],4), 'assoc', round(p['assoc_ms_per_frame'],4), 'integ', round(p['integrate_ms_per_frame'],4), 'render', round(p['render_ms_per_view'],4))" || exit 1
done
done
