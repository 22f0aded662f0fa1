#!/bin/bash
# per-rank cost of the N-GPU weak-scaling bench, one shard in one process
set -u
for cfg in "X=0" "BENCH_EMULATE_WORLD=2 BENCH_EMULATE_RANK=0" "BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=0" "BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=3" "BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=7"; do
  echo -n "[$cfg] "
  env $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pipeline --steps 20 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value'], 'kernel_ms', d['integrate_kernel_ms'], 'prep_ms', d['prep_ms'], 'step_ms', d['ms_per_step'], 'touched', d['touched_per_frame'], 'units', d['live_bricks_per_frame'])" || exit 1
done
