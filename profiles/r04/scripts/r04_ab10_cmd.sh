# r04: C4 strong-scaling emulation (8 ranks) at z-chunks 15, 31, 47; PC sampling probe of C3.
set -u
O=gpurun_out/r04_ab10
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1
echo "list rc=$?" >> $O/steps.log
for c in 47 31 15; do
  CHUNK=$c timeout -k 10 400 bash tools/emu_c4.sh gpurun_out/r04_ab10/emu_c$c "8" > $O/emu_c$c.txt 2>&1
  echo "emu $c rc=$?" >> $O/steps.log
done
