set -u
T=${1:-r05_final5}
bash tools/gpu_suite.sh $T/suite && bash tools/measure_final.sh $T && CHUNK=47 bash tools/emu_c4.sh gpurun_out/$T/c4emu 8 > gpurun_out/$T/c4emu.txt 2>&1 && tail -2 gpurun_out/$T/suite/pytest.log && cat gpurun_out/$T/c4emu.txt
