# r04: brick distance cap 12 / 16 (default) / 24 / 32 on the C3 pipeline (maps vs march trade).
set -u
O=gpurun_out/r04_ab26
mkdir -p $O
bash tools/ab_pipeline.sh build/var_cap24.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_cap32.so build/var_cap12.so build/var_cap24.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_cap32.so > $O/ab_cap.txt 2>&1
echo "ab rc=$?" >> $O/steps.log
