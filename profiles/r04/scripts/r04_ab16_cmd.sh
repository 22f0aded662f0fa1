# r04 combined: LPT on/off with the register tile sort, frame-set event skip vs the committed build,
# async prepass for the C3 step, fused/stream tests, pipeline kernel trace.
set -u
O=gpurun_out/r04_ab16
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "fused or async or stream" -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
for e in 1 0 1 0; do
  echo -n "[lpt=$e] " >> $O/ab_lpt.txt
  SEMTSDF_MARCH_LPT=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_lpt.txt 2>&1
  echo "lpt $e rc=$?" >> $O/steps.log
done
bash tools/ab_pipeline.sh build/var_head.so build/var_head.so >> $O/ab_lpt.txt 2>&1
echo "head rc=$?" >> $O/steps.log
for e in 1 0 1 0; do
  echo -n "[async=$e] " >> $O/ab_async.txt
  if [ $e = 1 ]; then AB_ARGS=--async-prepass bash tools/ab_integrate.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_async.txt 2>&1; else bash tools/ab_integrate.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_async.txt 2>&1; fi
  echo "async $e rc=$?" >> $O/steps.log
done
bash tools/trace_pipeline.sh r04_ab16/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
