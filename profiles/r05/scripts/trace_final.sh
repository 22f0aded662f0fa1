set -u
T=${1:-r05_trace}
O=gpurun_out/$T
mkdir -p $O
bash tools/trace_integrate.sh $O wtrace || exit 1
SEMTSDF_LIB=build/var_wtrace.so SEMTSDF_WAVE_TRACE=$O/trace_c2.bin timeout -k 10 300 python3 bench.py --only c2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
python3 tools/wave_trace.py $O/trace_c2.bin > $O/summary_c2.txt 2>&1; rm -f $O/trace_c2.bin
tail -17 $O/summary_wtrace.txt; tail -17 $O/summary_c2.txt
