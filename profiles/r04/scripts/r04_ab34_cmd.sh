# r04: frame prepass launched before the association (SEMTSDF_EARLY_PREP): fused/assoc tests on
# var_early.so (default on), pipeline A/B on/off, kernel trace with it on.
set -u
O=gpurun_out/r04_ab34
mkdir -p $O
SEMTSDF_LIB=$PWD/build/var_early.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_assoc_exact.py -k "fused or stream or exact or relabel or async or tum" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
for e in 1 0 1 0; do
  echo -n "[early=$e] " >> $O/ab_early.txt
  SEMTSDF_EARLY_PREP=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_early.txt 2>&1
  echo "e $e rc=$?" >> $O/steps.log
done
SEMTSDF_EARLY_PREP=1 bash tools/trace_pipeline.sh r04_ab34/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
