# r04: LPT launch order with the register-resident tile sort (on/off A/B), pipeline kernel trace.
set -u
O=gpurun_out/r04_ab14
mkdir -p $O
for e in 1 0 1 0; do
  echo -n "[lpt=$e] " >> $O/ab_lpt.txt
  SEMTSDF_MARCH_LPT=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_lpt.txt 2>&1
  echo "lpt $e rc=$?" >> $O/steps.log
done
bash tools/trace_pipeline.sh r04_ab14/trace_pipe > /dev/null 2>&1
echo "trace rc=$?" >> $O/steps.log
python3 tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
echo "timeline rc=$?" >> $O/steps.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "fused" -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
