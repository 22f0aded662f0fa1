set -u
mkdir -p gpurun_out/r04_ab4
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_assoc_exact.py -k "sharded" -v --timeout 200 --timeout-method thread > gpurun_out/r04_ab4/sharded.log 2>&1
echo "sharded rc=$?" >> gpurun_out/r04_ab4/steps.log
bash tools/ab_round4.sh r04_ab4
