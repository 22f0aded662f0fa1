# r04 end-of-round check on the final tree: GPU suite, smoke(), default bench line.
set -u
O=gpurun_out/r04_check2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
echo "suite rc=$?" >> $O/steps.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo "smoke rc=$?" >> $O/steps.log
timeout -k 10 700 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc=$?" >> $O/steps.log
