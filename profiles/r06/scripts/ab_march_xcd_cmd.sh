set -u
O=gpurun_out/r06_march_xcd; mkdir -p $O
SEMTSDF_LIB=$PWD/build/var_mx1.so timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "fused or bench_c3 or view or lpt or association_30" > $O/parity.txt 2>&1 || exit 1
for r in 1 2 3; do bash tools/ab_pipeline.sh build/var_mx0.so build/var_mx1.so >> $O/timing.txt 2>&1 || exit 1; done
