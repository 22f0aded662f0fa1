# r04: the frame's mask statistics + depth pyramid folded into the fused march launch
# (build/var_fold.so: SEMTSDF_FRAME_FOLD_DEFAULT=1): fused tests, pipeline A/B, kernel trace.
set -u
O=gpurun_out/r04_ab19
mkdir -p $O
SEMTSDF_LIB=$PWD/build/var_fold.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_assoc_exact.py -k "fused or stream or exact or relabel" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
bash tools/ab_pipeline.sh build/var_fold.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_fold.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > $O/ab_fold.txt 2>&1
echo "ab rc=$?" >> $O/steps.log
SEMTSDF_LIB=$PWD/build/var_fold.so bash tools/trace_pipeline.sh r04_ab19/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
