# r06: confirmation A/B of three frame sets (the new default) against the final two-set build (build/var_base.so):
# C3/C2 timing, the full bench line (pipeline, C4 single GPU), one emulated C4 rank; then the GPU suite on the new build
set -u
O=gpurun_out/r06_fs3; mkdir -p $O
AB_ROUNDS=3 AB_PMC=0 AB_C2=1 bash tools/ab_pmc.sh $O/ab build/var_base.so build/var_fs3main.so || exit 1
for r in 1 2; do
  for lib in build/var_base.so build/var_fs3main.so; do
    n=$(basename $lib .so)
    SEMTSDF_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    SEMTSDF_LIB=$lib BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=1 timeout -k 10 300 python3 bench.py --no-pipeline --no-cpu-baseline --steps 20 --c4-chunk 47 > $O/c4r1_${n}_$r.json 2> $O/c4r1_${n}_$r.err || exit 1
    echo "[fs3] $n round $r done" >> $O/steps.log
  done
done
bash tools/gpu_suite.sh r06_fs3/suite || exit 1
