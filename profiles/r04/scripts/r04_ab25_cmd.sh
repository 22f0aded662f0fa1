# r04: C4 8-rank emulation (async prepass) at z-chunk 15 (16-plane blocks: one cull unit each).
set -u
O=gpurun_out/r04_ab25
mkdir -p $O
CHUNK=15 timeout -k 10 600 bash tools/emu_c4.sh gpurun_out/r04_ab25/emu_c15 "8" > $O/emu_c15.txt 2>&1
echo "emu 15 rc=$?" >> $O/steps.log
