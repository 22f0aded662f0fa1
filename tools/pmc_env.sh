#!/bin/bash
# Instruction-mix PMC pass of the integrate bench under several environments (one rocprofv3
# run per environment, same counter set).  Usage:
#   bash tools/pmc_env.sh OUTDIR "COUNTERS" "ENV1=.. ENV2=.." "ENV3=.." ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; CTR=$2; shift 2
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-pipeline --steps 10 --warmup 2 --frames 4"}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 240 rocprofv3 --pmc $CTR --output-format csv -d $OUT/e$i -o run -- python3 $R/bench.py $ARGS > $OUT/e$i.log 2>&1
  rc=$?
  echo "env $i ($e) rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
