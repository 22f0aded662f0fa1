set -u
T=${1:-r05_s13}
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ids.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/first.log 2>&1 && \
AB_ARGS="--steps 40" bash tools/ab_integrate.sh build/rev_c2.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/rev_c2.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > gpurun_out/$T/ab.txt 2>&1 && \
for L in build/rev_c2.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so; do SEMTSDF_LIB=$L BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=0 timeout -k 10 120 python3 bench.py --no-pipeline --no-cpu-baseline --steps 20 --c4-chunk 47 > gpurun_out/$T/emu0.json 2>/dev/null && python3 -c "import json; d=json.load(open('gpurun_out/$T/emu0.json')); print('$L rank0', d['ms_per_step'], d['integrate_kernel_ms'])" >> gpurun_out/$T/ab.txt; done
