#!/bin/bash
# PMC passes of the integrate bench, one rocprofv3 run per quoted counter group.
# Usage: BENCH_ARGS="..." bash tools/pmc_groups.sh OUTDIR "CTR1 CTR2" "CTR3" ...   (env passes through)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
shift
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-pipeline --steps 10 --warmup 2 --frames 4"}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($ctr) rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
