#!/bin/bash
# Pipeline A/B (association + integrate frames/s, render): bash tools/_pipe_ab.sh "ENV=.." ...
set -u
for e in "$@"; do
  echo -n "[$e] "
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 30 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']
print('kernel_ms', d['integrate_kernel_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'], '| pipe fps %.1f assoc %.3f integ %.3f render %.3f' % (p['frames_per_s'], p['assoc_ms_per_frame'], p['integrate_ms_per_frame'], p['render_ms_per_view']))" || exit 1
done
