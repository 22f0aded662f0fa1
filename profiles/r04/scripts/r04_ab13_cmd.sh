# r04: maps computed ahead of the integrate (tests: conservative maps, fused == serial; pipeline
# A/B on/off), the faster tile order, GPU suite, pipeline kernel trace.
set -u
O=gpurun_out/r04_ab13
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_maps.py tests/test_gpu_parity.py -k "maps or fused" -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
for e in 1 0 1 0; do
  echo -n "[maps_ahead=$e] " >> $O/ab_ahead.txt
  SEMTSDF_MAPS_AHEAD=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_ahead.txt 2>&1
  echo "ahead $e rc=$?" >> $O/steps.log
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
echo "suite rc=$?" >> $O/steps.log
bash tools/trace_pipeline.sh r04_ab13/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
