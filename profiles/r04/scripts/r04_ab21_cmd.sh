# r04: decide ranks new labels over a compact list (tests + pipeline A/B vs the committed build
# var_head2 + kernel trace).
set -u
O=gpurun_out/r04_ab21
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_assoc_exact.py tests/test_gpu_parity.py -k "exact or fused or assoc or near or decision or relabel or label" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
bash tools/ab_pipeline.sh build/var_head2.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_head2.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > $O/ab_rank.txt 2>&1
echo "ab rc=$?" >> $O/steps.log
bash tools/trace_pipeline.sh r04_ab21/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
