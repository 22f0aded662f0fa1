# r04: C2 step with the async prepass vs in front (bench --only c2, --sync-prepass).
set -u
O=gpurun_out/r04_ab28
mkdir -p $O
for m in async sync async sync; do
  if [ $m = sync ]; then F=--sync-prepass; else F=; fi
  echo -n "[$m] " >> $O/ab_c2.txt
  timeout -k 10 200 python3 bench.py --only c2 $F 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d.get('c2', d); print('step', c['ms_per_step'], 'kernel', c['integrate_kernel_ms'], 'value', c['value'], 'frac', c['roofline']['frac'], c.get('prepass'))" >> $O/ab_c2.txt
  echo "$m rc=$?" >> $O/steps.log
done
