# r06: the C5 producer in fp16 with the box-size calibration: area probe, detector GPU tests, two masks-only bench lines
set -u
O=gpurun_out/${1:-r06_det_fp16}; mkdir -p $O
timeout -k 10 300 python3 tools/det_areas_probe.py > $O/areas_probe.txt 2> $O/areas_probe.err || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_maskrcnn.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/gputest_maskrcnn.txt 2>&1
echo "[det] tests rc=$?" >> $O/steps.log
grep -q "failed\|error" $O/gputest_maskrcnn.txt && exit 1
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --only masks --no-cpu-baseline > $O/bench_masks_$r.json 2> $O/bench_masks_$r.err || exit 1
  echo "[det] bench round $r" >> $O/steps.log
done
