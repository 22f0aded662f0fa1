# r04: decide phase timestamps (probe build var_dprobe.so, device printf) in the C3 pipeline.
set -u
O=gpurun_out/r04_ab29
mkdir -p $O
SEMTSDF_LIB=$PWD/build/var_dprobe.so timeout -k 10 300 python3 bench.py --only pipeline > $O/probe_out.txt 2> $O/probe_err.txt
echo "probe rc=$?" >> $O/steps.log
python3 - > $O/probe_summary.txt <<'PY'
import re, statistics as st
last, wg0 = [], []
for ln in open('gpurun_out/r04_ab29/probe_out.txt'):
    m = re.match(r'decide last wg (\d+) t0 (\d+) load\+cert (\d+) flags (\d+) wait (\d+) decide (\d+)', ln)
    if m: last.append([int(x) for x in m.groups()])
    m = re.match(r'decide wg0 t0 (\d+) load\+cert (\d+) flags (\d+) ticket (\d+)', ln)
    if m: wg0.append([int(x) for x in m.groups()])
print('last-arriver records', len(last), 'wg0 records', len(wg0))
if last:
    for i, name in enumerate(['wg', 't0', 'load+cert', 'flags', 'wait', 'decide']):
        if i >= 2: print(name, 'median ticks (10 ns)', st.median(r[i] for r in last))
    print('last wg ids (first 20)', [r[0] for r in last[:20]])
if wg0:
    for i, name in enumerate(['t0', 'load+cert', 'flags', 'ticket']):
        if i >= 1: print('wg0', name, 'median ticks', st.median(r[i] for r in wg0))
# last arriver t0 minus wg0 t0 (dispatch spread)
n = min(len(last), len(wg0))
print('last.t0 - wg0.t0 median ticks', st.median(last[i][1] - wg0[i][0] for i in range(n)) if n else None)
PY
echo "summary rc=$?" >> $O/steps.log
