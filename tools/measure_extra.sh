#!/bin/bash
# A round's second measurement call: the C4 per-rank emulation (8 ranks, 47-plane chunks), a
# 2-rank gloo rehearsal of the N > 1 bench on one GPU (both ranks share it: not scaling data),
# then the -m gpu suite and the smoke.  Usage: bash tools/measure_extra.sh TAG
set -u
TAG=${1:-extra}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
step() { echo "[extra] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
CHUNK=47 bash $R/tools/emu_c4.sh gpurun_out/$TAG/c4_emulation "8" > $O/c4_emulation.txt 2>&1
step c4_emulation $?
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err
step gloo_n2 $?
bash $R/tools/gpu_suite.sh $TAG/suite
step suite $?
