#!/bin/bash
# A round's closing GPU call: the -m gpu suite and the smoke, then the default bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-closing}
O=$R/gpurun_out/$TAG
mkdir -p $O
bash $R/tools/gpu_suite.sh $TAG/suite || exit 1
cd $R
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "[closing] bench rc=$?" | tee -a $O/steps.log
