# r04: speculative samples per evaluated sample (SEMTSDF_MARCH_SPEC 3 / 5 default / 7) on the
# fused pipeline.
set -u
O=gpurun_out/r04_ab31
mkdir -p $O
bash tools/ab_pipeline.sh build/var_spec3.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_spec7.so build/var_spec3.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_spec7.so > $O/ab_spec.txt 2>&1
echo "ab rc=$?" >> $O/steps.log
