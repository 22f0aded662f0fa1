#!/bin/bash
# PMC passes over a bench run.  Usage:
#   BENCH_ARGS="..." bash tools/pmc_integrate.sh OUTDIR "CTR1 CTR2" "CTR3" ...
# (one rocprofv3 run per quoted counter group; no trace domains are combined with --pmc)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/pmc}
shift
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-pipeline --steps 5 --warmup 1 --frames 4"}
i=0
for ctr in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($ctr) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
