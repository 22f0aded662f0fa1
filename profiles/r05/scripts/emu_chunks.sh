set -u
T=${1:-r05_emu_chunks}
for CH in 31 63; do
CHUNK=$CH bash tools/emu_c4.sh gpurun_out/$T/c$CH 8 > gpurun_out/$T/c$CH.txt 2>&1 || exit 1
done
cat gpurun_out/$T/c31.txt gpurun_out/$T/c63.txt
