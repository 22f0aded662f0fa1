# r04: frame-set events skipped when the prepass is ordered by the frame's entry event (in-tree)
# against the committed build (var_head); C3 step with the prepass beside the previous integrate.
set -u
O=gpurun_out/r04_ab15
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "fused or async or stream" -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
bash tools/ab_pipeline.sh build/var_head.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_head.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_head.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > $O/ab_setfree.txt 2>&1
echo "ab_setfree rc=$?" >> $O/steps.log
for e in 1 0 1 0 1 0; do
  echo -n "[async=$e] " >> $O/ab_async.txt
  if [ $e = 1 ]; then AB_ARGS=--async-prepass bash tools/ab_integrate.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_async.txt 2>&1; else bash tools/ab_integrate.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_async.txt 2>&1; fi
  echo "async $e rc=$?" >> $O/steps.log
done
