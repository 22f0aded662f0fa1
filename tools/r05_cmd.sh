set -u
T=${1:-r05_final4}
O=gpurun_out/$T
mkdir -p $O
bash tools/gpu_suite.sh $T/suite || exit 1
for rep in 1 2; do for lib in build/prev.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so; do
SEMTSDF_LIB=$lib timeout -k 10 200 python3 bench.py --only c2 --no-cpu-baseline > $O/c2ab.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/c2ab.json'))['c2']; print('c2 $lib', 'step', d['ms_per_step'], 'kernel', d['integrate_kernel_ms'], 'frac', d['roofline']['frac'])" >> $O/c2ab.txt
done; done
cat $O/c2ab.txt
bash tools/measure_final.sh $T && CHUNK=47 bash tools/emu_c4.sh gpurun_out/$T/c4emu 8 > gpurun_out/$T/c4emu.txt 2>&1 && tail -2 gpurun_out/$T/suite/pytest.log && cat gpurun_out/$T/c4emu.txt
