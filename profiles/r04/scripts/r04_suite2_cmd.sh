set -u
O=gpurun_out/r04_suite2
mkdir -p $O
bash tools/gpu_suite.sh r04_suite2 tests/test_gpu_assoc_exact.py
rc=$?
echo "suite rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --only pipeline > $O/pipe.json 2> $O/pipe.err
echo "pipe rc=$?" >> $O/steps.log
