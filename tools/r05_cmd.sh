set -u
T=${1:-r05_s11}
mkdir -p gpurun_out/$T
bash tools/gpu_suite.sh $T && \
timeout -k 10 900 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
