set -u
O=gpurun_out/r04_ab6
mkdir -p $O
bash tools/ab_pipeline.sh build/var_mp0.so build/var_mp8.so build/var_mp12.so build/var_mp20.so build/var_mp0.so build/var_mp8.so build/var_mp12.so build/var_mp20.so > $O/ab_pipe.txt 2>&1
echo "ab_pipe rc=$?" >> $O/steps.log
