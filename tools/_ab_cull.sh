#!/bin/bash
# Parity tests on the working lib, then same-box A/B of the working lib against build/var_base.so.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/ab
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -2 gpurun_out/ab/pytest.log
ROUNDS=${ROUNDS:-3} bash tools/_ab.sh "SEMTSDF_LIB=$R/build/var_base.so" "X=1"
