set -u
O=gpurun_out/r06_c2grid; mkdir -p $O
for r in 1 2; do
  for g in 0 2 3 4; do
    if [ $g = 0 ]; then unset SEMTSDF_GRID_PER_CU; else export SEMTSDF_GRID_PER_CU=$g; fi
    echo -n "grid_per_cu $g: " >> $O/c2.txt
    timeout -k 10 200 python3 bench.py --only c2 --no-cpu-baseline --steps 40 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['c2']
print('c2 kernel_ms', d['integrate_kernel_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'])" >> $O/c2.txt || exit 1
  done
done
unset SEMTSDF_GRID_PER_CU
