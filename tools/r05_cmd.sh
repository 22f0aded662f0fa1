set -u
T=${1:-r05_s16}
O=gpurun_out/$T
mkdir -p $O
for CH in 15 31; do
for r in 0 1 2 3 4 5 6 7; do
SEMTSDF_LIB=build/var_rr.so BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=$r timeout -k 10 120 python3 bench.py --no-pipeline --no-cpu-baseline --steps 20 --c4-chunk $CH > $O/c${CH}_r$r.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/c${CH}_r$r.json')); print('rr chunk $CH rank $r ms', d['ms_per_step'], 'kernel', d['integrate_kernel_ms'], 'live', d['live_units_per_frame'], 'free', d['free_units_per_frame'], 'touched', d['touched_per_frame'], 'gated', d['gated_per_frame'])" >> $O/summary.txt
done; done
