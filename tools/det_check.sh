#!/bin/bash
# GPU check of the Mask R-CNN producer: its tests, then the bench's producer leg alone.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-det}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_maskrcnn.py -x -v --timeout 500 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" | tee -a $O/steps.log
timeout -k 10 600 python3 bench.py --only masks > $O/masks.json 2> $O/masks.err
echo "bench rc=$?" | tee -a $O/steps.log
