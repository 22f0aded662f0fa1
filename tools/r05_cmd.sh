set -u
T=${1:-r05_s6}
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ids.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/first.log 2>&1 && \
AB_ARGS="--steps 40" bash tools/ab_integrate.sh build/rev_c1.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/rev_c1.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > gpurun_out/$T/ab.txt 2>&1
