set -u
T=${1:-r05_fix1s}
bash tools/gpu_suite.sh $T && tail -2 gpurun_out/$T/pytest.log && cat gpurun_out/$T/smoke.log | tail -1
