# r04 combined A/B (one box): cull variants (base = committed, soa1/soa2 = 16-byte tile-row loads
# with 1 or 2 units per lane), async prepass, LDS map passes (tests + pipeline A/B), ordering
# event flags, then the GPU suite on the in-tree library (soa2 cull, LPT, LDS maps).
set -u
O=gpurun_out/r04_ab11
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_maps.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/maps.log 2>&1
echo "maps rc=$?" >> $O/steps.log
bash tools/ab_integrate.sh build/var_base.so build/var_soa2.so build/var_soa1.so build/var_base.so build/var_soa2.so build/var_soa1.so > $O/ab_c3.txt 2>&1
echo "ab_c3 rc=$?" >> $O/steps.log
echo -n "[async] " >> $O/ab_async.txt
AB_ARGS=--async-prepass bash tools/ab_integrate.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_async.txt 2>&1
echo -n "[sync] " >> $O/ab_async.txt
bash tools/ab_integrate.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_async.txt 2>&1
echo "async rc=$?" >> $O/steps.log
for e in 0 1; do
  echo -n "[map_global=$e] " >> $O/ab_maps.txt
  SEMTSDF_MAP_GLOBAL=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_maps.txt 2>&1
  echo "maps $e rc=$?" >> $O/steps.log
done
for e in 1 2; do
  echo -n "[event_flags=$e] " >> $O/ab_maps.txt
  SEMTSDF_EVENT_FLAGS=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_maps.txt 2>&1
  echo "events $e rc=$?" >> $O/steps.log
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
echo "suite rc=$?" >> $O/steps.log
