for g in 5 4 3 2 1 5 3 2; do
  echo -n "grid_per_cu $g: "
  SEMTSDF_GRID_PER_CU=$g timeout -k 10 200 python3 bench.py --only c2 --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['c2']; print(d['integrate_kernel_ms'], d['ms_per_step'], d['touched_mvox_per_s'])" || exit 1
done
