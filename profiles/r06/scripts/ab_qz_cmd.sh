# r06: A/B of the quarter-step zero-threshold brick skip (SEMTSDF_QUARTER_ZERO, build/var_qz.so) against the
# final build (build/var_base.so): march/association/render/integrate parity on var_qz, then the live pipeline and
# orbit (bench --only pipeline), C3 integrate timing, 3 interleaved rounds
set -u
O=gpurun_out/r06_qz; mkdir -p $O
SEMTSDF_LIB=build/var_qz.so timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
  -k "march or render or assoc or fused or bench_config or parse_frame or integrate_bit_exact or full_size_512 or map or oct or skip" > $O/parity.txt 2>&1
echo "[qz] parity rc=$?" >> $O/steps.log; tail -1 $O/parity.txt >> $O/steps.log
grep -q " passed" $O/parity.txt && ! grep -q "failed\|error" $O/parity.txt || exit 1
for r in 1 2 3; do
  for lib in build/var_base.so build/var_qz.so; do
    n=$(basename $lib .so)
    SEMTSDF_LIB=$lib timeout -k 10 300 python3 bench.py --only pipeline --no-cpu-baseline > $O/pipe_${n}_$r.json 2> $O/pipe_${n}_$r.err || exit 1
    echo "[qz] $n round $r" >> $O/steps.log
  done
  bash tools/ab_integrate.sh build/var_base.so build/var_qz.so > $O/timing_round$r.txt 2>&1 || exit 1
done
