# A/B: unit cull with 16-byte tile-row loads from the padded SoA pyramid levels, one (soa1) or
# two (soa2) units per lane, against the committed cull (base); async prepass with soa2.
set -u
O=gpurun_out/r04_ab8
mkdir -p $O
SEMTSDF_LIB=$PWD/build/var_soa2.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_soa2.log 2>&1
echo "parity rc=$?" >> $O/steps.log
bash tools/ab_integrate.sh build/var_base.so build/var_soa2.so build/var_soa1.so build/var_base.so build/var_soa2.so build/var_soa1.so > $O/ab_c3.txt 2>&1
echo "ab_c3 rc=$?" >> $O/steps.log
for g in 1 0 1 0; do
  echo -n "[async=$g] " >> $O/ab_async.txt
  if [ $g = 1 ]; then AB_ARGS=--async-prepass bash tools/ab_integrate.sh build/var_soa2.so >> $O/ab_async.txt 2>&1; else bash tools/ab_integrate.sh build/var_soa2.so >> $O/ab_async.txt 2>&1; fi
  echo "async $g rc=$?" >> $O/steps.log
done
for lib in build/var_base.so build/var_soa2.so build/var_base.so build/var_soa2.so; do
  echo -n "[$lib] " >> $O/ab_c2.txt
  SEMTSDF_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --only c2 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d.get('c2', d); print('kernel', c['integrate_kernel_ms'], 'step', c['ms_per_step'], 'frac', c['roofline']['frac'])" >> $O/ab_c2.txt
  echo "c2 rc=$?" >> $O/steps.log
done
