set -u
T=${1:-r05_fs3}
O=gpurun_out/$T
mkdir -p $O
SEMTSDF_LIB=build/var_fs3.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "async or pipeline or fused" -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
bash tools/ab_integrate.sh build/rev_head.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_fs3.so build/rev_head.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_fs3.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
