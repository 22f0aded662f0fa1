set -u
O=gpurun_out/r06_nts; mkdir -p $O
for r in 1 2 3 4; do bash tools/ab_integrate.sh build/var_base.so build/var_ntstore0.so >> $O/timing.txt 2>&1 || exit 1; done
for r in 1 2; do bash tools/ab_pipeline.sh build/var_base.so build/var_ntstore0.so >> $O/pipeline.txt 2>&1 || exit 1; done
