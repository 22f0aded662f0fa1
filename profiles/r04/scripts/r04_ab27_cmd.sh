# r04: host-copy kernel (pinned -> HBM uploads beside the volume's kernels): old 64-workgroup
# one-read copy vs unrolled copy on 8 / 16 / 32 workgroups; copy test.
set -u
O=gpurun_out/r04_ab27
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "pinned or memcpy or copy" -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
for w in 0 16 8 32 0 16; do
  echo -n "[copy_wgs=$w] " >> $O/ab_copy.txt
  SEMTSDF_COPY_HOST_WGS=$w bash tools/ab_pipeline.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so >> $O/ab_copy.txt 2>&1
  echo "w $w rc=$?" >> $O/steps.log
done
