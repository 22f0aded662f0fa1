"""Where a bench step goes beyond its integrate kernel (rocprofv3 --kernel-trace of a bench run
with the prepass beside the previous integrate): per consecutive pair of integrate dispatches,
the interval between their starts, the first one's duration, and the next frame's prepass
kernels (depth pyramid, cull) relative to the first integrate's end.  Medians over the trace.
Usage: python tools/step_gaps.py TRACE_DIR [integrate_kernel_substring]"""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
ik = sys.argv[2] if len(sys.argv) > 2 else "k_integrate<true, true, false, false, false, false, true>"
rows = []
for fn in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
ints = [r for r in rows if ik in r[2]]
pyr = [r for r in rows if "k_depth_pyramid" in r[2]]
cull = [r for r in rows if "k_cull_units" in r[2]]
stats = {k: [] for k in ("interval", "integrate", "end_to_next_start", "pyr_start_rel_end", "pyr_dur",
                         "cull_start_rel_end", "cull_end_rel_end", "cull_dur")}
for a, b in zip(ints, ints[1:]):
    iv = (b[0] - a[0]) / 1e3
    if iv > 400:  # a pass boundary (host work between the bench's passes)
        continue
    stats["interval"].append(iv)
    stats["integrate"].append((a[1] - a[0]) / 1e3)
    stats["end_to_next_start"].append((b[0] - a[1]) / 1e3)
    # the prepass feeding b: the last pyramid / cull that started before b
    p = [r for r in pyr if r[0] < b[0] and r[0] > a[0] - 200e3]
    c = [r for r in cull if r[0] < b[0] and r[0] > a[0] - 200e3]
    if p:
        stats["pyr_start_rel_end"].append((p[-1][0] - a[1]) / 1e3)
        stats["pyr_dur"].append((p[-1][1] - p[-1][0]) / 1e3)
    if c:
        stats["cull_start_rel_end"].append((c[-1][0] - a[1]) / 1e3)
        stats["cull_end_rel_end"].append((c[-1][1] - a[1]) / 1e3)
        stats["cull_dur"].append((c[-1][1] - c[-1][0]) / 1e3)
print(f"{len(ints)} integrate dispatches, {len(stats['interval'])} consecutive pairs")
for k, v in stats.items():
    if v:
        q = sorted(v)
        print(f"{k:22s} median {statistics.median(v):8.2f} us  p10 {q[len(q) // 10]:8.2f}  p90 {q[9 * len(q) // 10]:8.2f}")
