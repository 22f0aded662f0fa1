"""One-line summary of a bench.py JSON line on stdin (integrate timing and work counts)."""
import json
import sys

d = json.loads(sys.stdin.read())
print('kernel_ms', d['integrate_kernel_ms'], 'prep_ms', d['prep_ms'], 'step_ms', d['ms_per_step'], 'touched',
      d['touched_per_frame'], 'units', d['live_bricks_per_frame'])
