#!/bin/bash
# GPU: detector tests + producer bench leg, then rocprofv3 kernel stats of the producer leg.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-det_prof}
bash $R/tools/det_check.sh $TAG || exit 1
O=$R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --only masks > $O/masks_prof.json 2> $O/masks_prof.err
echo "prof rc=$?" | tee -a $O/steps.log
