# r04: ordering-event flags A/B (0: system-scope release, 2: no system fence) and LPT on/off on
# the in-tree library; GPU suite; C4 strong-scaling emulation at z-chunks 47 and 23.
set -u
O=gpurun_out/r04_ab12
mkdir -p $O
for e in 0 2 0 2; do
  echo -n "[event_flags=$e] " >> $O/ab_events.txt
  SEMTSDF_EVENT_FLAGS=$e bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_events.txt 2>&1
  echo "events $e rc=$?" >> $O/steps.log
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
echo "suite rc=$?" >> $O/steps.log
for c in 47 23; do
  CHUNK=$c timeout -k 10 400 bash tools/emu_c4.sh gpurun_out/r04_ab12/emu_c$c "8" > $O/emu_c$c.txt 2>&1
  echo "emu $c rc=$?" >> $O/steps.log
done
