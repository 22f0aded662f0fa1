# r04: map passes through LDS (tests + pipeline A/B against the global passes), LPT on/off,
# then the GPU suite on the in-tree library.
set -u
O=gpurun_out/r04_ab9
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_maps.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/maps.log 2>&1
echo "maps rc=$?" >> $O/steps.log
for e in 0 1 0 1; do
  echo -n "[map_global=$e] " >> $O/ab_maps.txt
  SEMTSDF_MAP_GLOBAL=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_maps.txt 2>&1
  echo "maps $e rc=$?" >> $O/steps.log
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
echo "suite rc=$?" >> $O/steps.log
for e in 0 1 2 0 1 2; do
  echo -n "[event_flags=$e] " >> $O/ab_events.txt
  SEMTSDF_EVENT_FLAGS=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_events.txt 2>&1
  echo "events $e rc=$?" >> $O/steps.log
done
