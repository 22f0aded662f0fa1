#!/bin/bash
# Final measurement of a round in one call: PMC traffic + counters of C3 and C2 (stamped with the build
# key), the traffic records copied where bench.py reads them, the bench line, rocprofv3 kernel
# stats of the C3 bench, a kernel trace of the fused pipeline and of one C4 emulated rank.
set -u
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "[measure] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
bash $R/tools/measure_pmc.sh $TAG
step partA $?
cp $O/traffic.json $R/profiles/traffic_latest.json && cp $O/c2/traffic.json $R/profiles/traffic_c2_latest.json
step copy_traffic $?
bash $R/tools/measure_bench.sh $TAG
step partB $?
bash $R/tools/trace_pipeline.sh $TAG/trace_pipe > /dev/null 2>&1
step trace_pipe $?
python3 $R/tools/timeline.py $O/trace_pipe/trace 40 3 k_march_fused > $O/timeline_pipe.txt 2>&1
step timeline_pipe $?
cd /tmp && export TMPDIR=/tmp
BENCH_EMULATE_WORLD=8 BENCH_EMULATE_RANK=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c4r1 -o run -- python3 $R/bench.py --no-pipeline --no-cpu-baseline --steps 20 --c4-chunk 47 > $O/c4r1.json 2> $O/c4r1.err
step trace_c4r1 $?
python3 $R/tools/timeline.py $O/trace_c4r1 12 3 k_depth_pyramid > $O/timeline_c4r1.txt 2>&1
step timeline_c4r1 $?
