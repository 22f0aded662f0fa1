set -u
T=${1:-r05_s4}
mkdir -p gpurun_out/$T
bash tools/gpu_suite.sh $T && \
AB_ARGS="--steps 40" bash tools/ab_integrate.sh build/rev_r04.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/rev_r04.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > gpurun_out/$T/ab.txt 2>&1
