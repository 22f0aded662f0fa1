# r06: the HIP ROI align in the C5 producer: detector GPU tests, two masks-only bench lines, producer kernel stats
set -u
O=gpurun_out/${1:-r06_det_roi}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_maskrcnn.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/gputest_maskrcnn.txt 2>&1
echo "[det] tests rc=$?" >> $O/steps.log
grep -q "failed\|error" $O/gputest_maskrcnn.txt && exit 1
timeout -k 10 300 python3 tools/det_areas_probe.py > $O/areas_probe.txt 2> $O/areas_probe.err || exit 1
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --only masks --no-cpu-baseline > $O/bench_masks_$r.json 2> $O/bench_masks_$r.err || exit 1
  echo "[det] bench round $r" >> $O/steps.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --only masks --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/masks_prof.json 2> $GRAFT_REPO_ROOT/$O/masks_prof.err
echo "[det] prof rc=$?" >> $GRAFT_REPO_ROOT/$O/steps.log
