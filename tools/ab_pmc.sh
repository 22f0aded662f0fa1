#!/bin/bash
# Same-box A/B of library builds: parity subset on the last build, C3 timing (interleaved rounds),
# then PMC FETCH_SIZE / WRITE_SIZE of the C3 integrate per build.
# Usage: bash tools/ab_pmc.sh OUTDIR LIB1.so LIB2.so ...   (AB_ROUNDS, AB_TESTS, AB_PMC=0 to skip)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; shift
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[ab] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
LAST=${@: -1}
if [ -n "${AB_TESTS:-}" ]; then
  SEMTSDF_LIB=$R/$LAST timeout -k 10 600 python3 -u -m pytest $R/tests -x -q -m gpu --timeout 300 --timeout-method thread \
    -k "${AB_TESTS}" > $O/parity.txt 2>&1
  step "parity $LAST" $?
fi
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  bash $R/tools/ab_integrate.sh "$@" > $O/timing_round$r.txt 2>&1
  step "timing round $r" $?
  if [ "${AB_C2:-0}" = "1" ]; then
    for lib in "$@"; do
      echo -n "[$lib] " >> $O/timing_c2_round$r.txt
      SEMTSDF_LIB=$R/$lib timeout -k 10 200 python3 $R/bench.py --only c2 --no-cpu-baseline --steps 40 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['c2']
print('c2 kernel_ms', d['integrate_kernel_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'])" >> $O/timing_c2_round$r.txt
      step "c2 timing $lib round $r" $?
    done
  fi
done
if [ "${AB_PMC:-1}" = "1" ]; then
  cd /tmp
  for lib in "$@"; do
    n=$(basename $lib .so)
    for c in FETCH_SIZE WRITE_SIZE; do
      SEMTSDF_LIB=$R/$lib timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${n}_$c -o run -- \
        python3 $R/bench.py --no-cpu-baseline --no-pipeline --no-c4 --steps 10 --warmup 2 --frames 4 > $O/pmc_${n}_$c.json 2> $O/pmc_${n}_$c.err
      step "pmc $n $c" $?
    done
  done
fi
