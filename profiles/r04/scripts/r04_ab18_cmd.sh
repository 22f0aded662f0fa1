# r04: bench upload ring with HIP events (no system fence) vs torch events; C4 8-rank emulation
# with the async prepass (bench default now); rocprofv3 PC-sampling capabilities.
set -u
O=gpurun_out/r04_ab18
mkdir -p $O
for e in 1 0 1 0; do
  echo -n "[hip_events=$e] " >> $O/ab_events.txt
  BENCH_HIP_EVENTS=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_events.txt 2>&1
  echo "ev $e rc=$?" >> $O/steps.log
done
CHUNK=47 timeout -k 10 500 bash tools/emu_c4.sh gpurun_out/r04_ab18/emu_c47 "8" > $O/emu_c47.txt 2>&1
echo "emu rc=$?" >> $O/steps.log
timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1
echo "list rc=$?" >> $O/steps.log
