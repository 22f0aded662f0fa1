# r04: sharded async-prepass test; C4 8-rank emulation (async prepass) at z-chunks 31 and 63.
set -u
O=gpurun_out/r04_ab24
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "async" -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
for c in 31 63; do
  CHUNK=$c timeout -k 10 500 bash tools/emu_c4.sh gpurun_out/r04_ab24/emu_c$c "8" > $O/emu_c$c.txt 2>&1
  echo "emu $c rc=$?" >> $O/steps.log
done
