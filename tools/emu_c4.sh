#!/bin/bash
# Per-rank cost of the C4 strong-scaling integrate (one rank's shard of the 1024^3 volume in
# one process; bench.py BENCH_EMULATE_WORLD/RANK): bash tools/emu_c4.sh OUTDIR "2 4 8"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; mkdir -p $O
for w in $2; do
  for r in ${RANKS:-$(seq 0 $((w - 1)))}; do
    BENCH_EMULATE_WORLD=$w BENCH_EMULATE_RANK=$r timeout -k 10 120 python3 $R/bench.py --no-pipeline --no-cpu-baseline --steps 20 --c4-chunk ${CHUNK:-64} ${EMU_ARGS:-} > $O/w${w}_r${r}.json 2> $O/w${w}_r${r}.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/w${w}_r${r}.json')); print('world $w rank $r ms_per_step', d['ms_per_step'], 'kernel', d['integrate_kernel_ms'], 'prep', d['prep_ms'], 'touched', d['touched_per_frame'])"
  done
done
