# quick integrate timing (kernel + prep) at 512^3; extra args are passed to bench.py
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pipeline --steps 20 "$@" 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value'], 'kernel_ms', d['integrate_kernel_ms'], 'prep_ms', d['prep_ms'], 'step_ms', d['ms_per_step'], 'bricks', d['live_units_per_frame'], 'frac', d['roofline']['frac'])"
