#!/bin/bash
# r04 A/B on one box: per-lane vs whole-line state traffic (parity + C3/C2 timing), and the
# pipeline with the relabel folded into the integrate vs the separate relabel kernel.
# Usage: bash tools/ab_round4.sh TAG   (libraries prebuilt under build/)
set -u
TAG=${1:-ab4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
step() { echo "[ab4] $1 rc=$2" | tee -a $O/steps.log; if [ $2 -ne 0 ]; then exit $2; fi; }
SEMTSDF_LIB=$R/build/var_perlane.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_perlane.log 2>&1
step parity_perlane $?
bash tools/ab_integrate.sh build/var_fullrow.so build/var_perlane.so build/var_fullrow.so build/var_perlane.so > $O/ab_c3.txt 2>&1
step ab_c3 $?
for lib in build/var_fullrow.so build/var_perlane.so build/var_fullrow.so build/var_perlane.so; do
  echo -n "[$lib] " >> $O/ab_c2.txt
  SEMTSDF_LIB=$R/$lib timeout -k 10 200 python3 bench.py --only c2 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d.get('c2', d); print(json.dumps(c)[:600])" >> $O/ab_c2.txt
  step c2 $?
done
for rk in 1 0 1 0; do
  echo -n "[relabel_kernel=$rk] " >> $O/ab_pipe.txt
  SEMTSDF_RELABEL_KERNEL=$rk SEMTSDF_LIB=$R/build/var_perlane.so timeout -k 10 300 python3 bench.py --only pipeline 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['pipeline']; p=d['pipeline']
print('fps %.1f serial %.1f exact_frames %s/%s all_exact_fps %.1f assoc %.4f integ %.4f' % (p['frames_per_s'], p['serial_frames_per_s'], p['assoc_exact_frames'], p['assoc_decisions'], p['all_exact_frames_per_s'], p['assoc_ms_per_frame'], p['integrate_ms_per_frame']))" >> $O/ab_pipe.txt
  step pipe $?
done
bash tools/trace_integrate.sh gpurun_out/$TAG/wtrace wtrace > $O/wtrace.log 2>&1
step wtrace $?
