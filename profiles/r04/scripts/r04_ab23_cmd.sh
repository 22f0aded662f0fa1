# r04: render launch order (SEMTSDF_RENDER_LPT) on/off: render/raycast tests, pipeline (serial +
# orbit views) A/B.
set -u
O=gpurun_out/r04_ab23
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
echo "suite rc=$?" >> $O/steps.log
for e in 1 0 1 0; do
  echo -n "[render_lpt=$e] " >> $O/ab_render.txt
  SEMTSDF_RENDER_LPT=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_render.txt 2>&1
  echo "r $e rc=$?" >> $O/steps.log
done
