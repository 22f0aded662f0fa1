#!/bin/bash
# PMC byte calibration (tools/membench_calib.hip) and the split of k_integrate's fetched bytes into
# its state traffic and the rest (probe build, SEMTSDF_DEBUG_INTEGRATE=3: no state traffic).
# Needs build/membench_calib and build/var_probes.so (tools/build_variant.sh probes
# -DSEMTSDF_INTEGRATE_PROBES=1).  Usage: bash tools/calib_pmc.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/calib}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
step() { echo "[calib] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 60 $R/build/membench_calib 5 > $O/known.jsonl 2> $O/known.err
step timing $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $R/build/membench_calib 2 > $O/fetch.log 2>&1
step fetch $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $R/build/membench_calib 2 > $O/write.log 2>&1
step write $?
python3 $R/tools/calib_summary.py $O/known.jsonl $O/fetch $O/write $O/calibration.json > $O/calibration.txt 2>&1
step summary $?
ARGS="--no-cpu-baseline --no-pipeline --no-c4 --steps 10 --warmup 2 --frames 4"
for m in 0 3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SEMTSDF_LIB=$R/build/var_probes.so SEMTSDF_DEBUG_INTEGRATE=$m timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv \
      -d $O/probe_m${m}_$c -o run -- python3 $R/bench.py $ARGS > $O/probe_m${m}_$c.json 2> $O/probe_m${m}_$c.err
    step "probe mode $m $c" $?
  done
done
