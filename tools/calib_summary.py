"""PMC byte calibration per access pattern (tools/membench_calib.hip).

Joins the known byte counts membench_calib prints (one JSON object per kernel) with the
FETCH_SIZE / WRITE_SIZE rows of two rocprofv3 --pmc passes over the same program, and writes
per-pattern factors: bytes = factor x counter bytes (FETCH_SIZE in KiB x 1024).
Usage: python tools/calib_summary.py KNOWN_JSONL FETCH_PASS_DIR WRITE_PASS_DIR OUT_JSON
"""
import collections
import csv
import glob
import json
import sys


def counter_means(d, name):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                k = r["Kernel_Name"].split("(")[0].strip()
                vals[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    known = [json.loads(ln) for ln in open(sys.argv[1]) if ln.startswith("{")]
    fetch = counter_means(sys.argv[2], "FETCH_SIZE")
    write = counter_means(sys.argv[3], "WRITE_SIZE")
    rows = []
    for k in known:
        name = k["kernel"]
        fb = next((v for n, v in fetch.items() if n.endswith(name)), None)
        wb = next((v for n, v in write.items() if n.endswith(name)), None)
        row = dict(k)
        row["fetch_size_bytes"] = fb
        row["write_size_bytes"] = wb
        row["fetch_factor"] = (k["known_read"] / fb) if fb and k["known_read"] else None
        row["write_factor"] = (k["known_write"] / wb) if wb and k["known_write"] else None
        rows.append(row)
        print(f"{name:18s} known r {k['known_read'] / 1e6:9.2f} MB  FETCH_SIZE {fb / 1e6 if fb else float('nan'):9.2f} MB"
              f"  -> x{row['fetch_factor'] or float('nan'):.3f}   known w {k['known_write'] / 1e6:8.2f} MB"
              f"  WRITE_SIZE {wb / 1e6 if wb else float('nan'):8.2f} MB -> x{row['write_factor'] or float('nan'):.3f}"
              f"   {k['us']:.1f} us {k['gbs']:.0f} GB/s")
    json.dump({"source": "tools/membench_calib.hip + rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes)",
               "rows": rows}, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
