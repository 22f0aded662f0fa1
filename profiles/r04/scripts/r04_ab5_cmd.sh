set -u
O=gpurun_out/r04_ab5
mkdir -p $O
step() { echo "[ab5] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_assoc_exact.py -k "sharded" -v --timeout 200 --timeout-method thread > $O/sharded.log 2>&1
echo "[ab5] sharded rc=$?" >> $O/steps.log
bash tools/ab_integrate.sh build/var_noprio.so build/var_prio.so build/var_noprio.so build/var_prio.so > $O/ab_c3.txt 2>&1
step ab_c3 $?
bash tools/trace_integrate.sh $O/wtrace wtrace > $O/wtrace.log 2>&1
step wtrace $?
bash tools/ab_pipeline.sh build/var_noprio.so build/var_prio.so > $O/ab_pipe.txt 2>&1
step ab_pipe $?
