#!/bin/bash
# Per-rank cost of one shard for several z_chunk values: bash tools/_emu_chunk.sh "31 32 63"
set -u
for c in ${1:-31 32}; do
for cfg in "BENCH_EMULATE_WORLD=2 BENCH_EMULATE_RANK=0" "BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=0" "BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=7"; do
  echo -n "[chunk $c $cfg] "
  env $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pipeline --steps 20 --z-chunk $c 2>/dev/null | python3 tools/_bench_summary.py || exit 1
done
done
