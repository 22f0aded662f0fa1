set -u
T=${1:-r05_prio}
O=gpurun_out/$T
mkdir -p $O
bash tools/ab_integrate.sh slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_prio2.so build/var_prio8.so slam-maskrcnn_amd/semtsdf/libsemtsdf.so build/var_prio2.so build/var_prio8.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
