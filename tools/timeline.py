"""Timeline of a rocprofv3 kernel trace (tools/trace_pipeline.sh): per k_assoc_march-started
frame, the kernels in order with durations and the idle gaps between them.
Usage: python tools/timeline.py TRACE_DIR [first_frame] [n_frames] [frame_kernel]
(frame_kernel: the kernel that starts a frame, default k_assoc_march; k_march_fused for the
fused pipeline)"""
import csv
import glob
import re
import sys

d = sys.argv[1]
f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 20
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 3
fk = sys.argv[4] if len(sys.argv) > 4 else "k_assoc_march"
rows = []
for fn in glob.glob(f"{d}/*kernel_trace.csv"):
    for r in csv.DictReader(open(fn)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], "K"))
for fn in glob.glob(f"{d}/*memory_copy_trace.csv"):
    for r in csv.DictReader(open(fn)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "copy"), "C"))
rows.sort()
def short(n):
    n = re.sub(r"\(.*", "", n)
    return n.replace("semtsdf::", "")[:60]
starts = [i for i, r in enumerate(rows) if fk in r[2]]
print(f"{len(starts)} frames ({fk})")
tot_busy = tot_span = 0.0
for fi in range(f0, min(f0 + nf, len(starts) - 1)):
    a, b = starts[fi], starts[fi + 1]
    span = (rows[b][0] - rows[a][0]) / 1e3
    busy = 0.0
    prev_end = rows[a][0]
    print(f"--- frame {fi}: span {span:.1f} us")
    for s, e, n, k in rows[a:b]:
        if k == "C":
            print(f"   [copy {n}] {(e - s) / 1e3:7.1f} us")
            continue
        gap = (s - prev_end) / 1e3
        busy += (e - s) / 1e3
        print(f"  gap {gap:6.1f}  {short(n):60s} {(e - s) / 1e3:7.1f} us")
        prev_end = max(prev_end, e)
    print(f"   busy {busy:.1f} us of {span:.1f}")
