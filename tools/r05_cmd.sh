set -u
T=${1:-r05_spec}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ab_integrate.sh build/prev.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/prev.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/prev.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
