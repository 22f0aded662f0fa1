# r04: decide without hand-off fences when no row is flagged, tile order in its own workgroup:
# exact-path tests, fused tests, pipeline A/B against the committed build, kernel trace.
set -u
O=gpurun_out/r04_ab17
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_assoc_exact.py tests/test_gpu_parity.py -k "exact or fused or assoc or near or decision" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
bash tools/ab_pipeline.sh build/var_head.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_head.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_fwpe5.so > $O/ab_decide.txt 2>&1
echo "ab rc=$?" >> $O/steps.log
bash tools/trace_pipeline.sh r04_ab17/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
