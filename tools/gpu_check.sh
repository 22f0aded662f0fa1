#!/bin/bash
# GPU-box check: parity tests, smoke, one bench line.  Usage: bash tools/gpu_check.sh TAG [bench args]
set -u
TAG=${1:-check}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
step() { echo "[check] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step pytest $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step smoke $?
timeout -k 10 300 python3 bench.py "$@" > $O/bench.json 2> $O/bench.err
step bench $?
cat $O/bench.json
