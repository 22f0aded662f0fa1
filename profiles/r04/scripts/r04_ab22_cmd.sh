# r04: decide with its table loads hoisted (and the frame-fold instrumentation bit): GPU suite,
# pipeline A/B against the committed build (var_head3), kernel trace.
set -u
O=gpurun_out/r04_ab22
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
echo "suite rc=$?" >> $O/steps.log
bash tools/ab_pipeline.sh build/var_head3.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_head3.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > $O/ab_decide.txt 2>&1
echo "ab rc=$?" >> $O/steps.log
bash tools/trace_pipeline.sh r04_ab22/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
