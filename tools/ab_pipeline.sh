#!/bin/bash
# Same-box A/B of library builds on the C3 pipeline section (association + integrate +
# render per frame, then the orbit views): bash tools/ab_pipeline.sh LIB1.so LIB2.so ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$@"; do
  echo -n "[$lib] "
  SEMTSDF_LIB=$R/$lib timeout -k 10 200 python3 $R/bench.py --only pipeline 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['pipeline']; p=d['pipeline']; o=d['orbit']
print('serial %.1f ovl %.1f fps %.1f assoc %.4f integ %.4f render %.4f | orbit views/s %.1f render %.4f | equal %s %s' % (p['serial_frames_per_s'], p['overlapped_frames_per_s'], p['frames_per_s'], p['assoc_ms_per_frame'], p['integrate_ms_per_frame'], p['render_ms_per_view'], o['views_per_s'], o['render_ms_per_view'], p.get('fused_equals_serial'), p.get('overlapped_equals_serial')))" || exit 1
done
