set -u
T=${1:-r05_dyn4}
O=gpurun_out/$T
mkdir -p $O
AB_ARGS=--no-c4 bash tools/ab_integrate.sh build/var_noopt.so build/var_dyn_s8.so build/var_dyn_s32.so build/var_noopt.so build/var_dyn_s8.so build/var_dyn_s32.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
