set -u
CHUNK=47 bash tools/emu_c4.sh gpurun_out/r06_emu2 "8" > gpurun_out/r06_emu2.txt 2>&1 || exit 1
