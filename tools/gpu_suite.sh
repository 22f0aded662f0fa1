#!/bin/bash
# GPU-box check of a change: the named test files first, then the whole -m gpu suite and the
# smoke.  Usage: bash tools/gpu_suite.sh TAG [test files...]
set -u
TAG=${1:-suite}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
step() { echo "[suite] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
if [ $# -gt 0 ]; then
  timeout -k 10 600 python3 -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $O/first.log 2>&1
  step first $?
fi
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
step pytest $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step smoke $?
