# A/B: unit cull with two units per lane (build/var_cull2.so) vs the committed cull
# (build/var_base.so); the prepass on the prep stream beside the previous integrate with the
# integrate's persistent grid at 3 or 4 workgroups per CU.
set -u
O=gpurun_out/r04_ab7
mkdir -p $O
SEMTSDF_LIB=$PWD/build/var_cull2.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_cull2.log 2>&1
echo "parity rc=$?" >> $O/steps.log
bash tools/ab_integrate.sh build/var_base.so build/var_cull2.so build/var_base.so build/var_cull2.so > $O/ab_c3.txt 2>&1
echo "ab_c3 rc=$?" >> $O/steps.log
for g in 4 3 4 3; do
  echo -n "[async grid_per_cu=$g] " >> $O/ab_async.txt
  SEMTSDF_GRID_PER_CU=$g AB_ARGS=--async-prepass bash tools/ab_integrate.sh build/var_cull2.so >> $O/ab_async.txt 2>&1
  echo "async $g rc=$?" >> $O/steps.log
done
for g in 3; do
  echo -n "[sync grid_per_cu=$g] " >> $O/ab_async.txt
  SEMTSDF_GRID_PER_CU=$g bash tools/ab_integrate.sh build/var_cull2.so >> $O/ab_async.txt 2>&1
  echo "sync $g rc=$?" >> $O/steps.log
done
SEMTSDF_LIB=$PWD/build/var_lpt.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_assoc_exact.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_lpt.log 2>&1
echo "tests_lpt rc=$?" >> $O/steps.log
for e in 0 1 0 1; do
  echo -n "[lpt=$e] " >> $O/ab_lpt.txt
  SEMTSDF_MARCH_LPT=$e bash tools/ab_pipeline.sh build/var_lpt.so >> $O/ab_lpt.txt 2>&1
  echo "lpt $e rc=$?" >> $O/steps.log
done
