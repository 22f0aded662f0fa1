"""Per-launch HBM bytes of one kernel from rocprofv3 PMC passes (tools/pmc_integrate.sh).

FETCH_SIZE and WRITE_SIZE (KiB) are collected in separate passes (they do not fit one TCC
pass on gfx950).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports half the bytes of wide
coalesced reads on gfx950, so it is doubled; WRITE_SIZE is taken as is.
The record is stamped with the SHA-256 of the library whose kernel was profiled
(SEMTSDF_LIB or the in-tree libsemtsdf.so): bench.py reports the traffic only when the
library it loads has the same hash.
Usage: python tools/traffic.py PMC_DIR KERNEL_SUBSTRING OUT_JSON DIM [N_GPUS]
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# known-byte record of the correction for the integrate's own access patterns (tools/membench_calib.hip,
# tools/calib_pmc.sh): x2 holds for 16-B, 8-B and 4-B loads and line-distinct 8-B gathers; x1 for
# 16-B non-temporal stores
CALIBRATION = "profiles/r06/calib/calibration.json"


def lib_sha256(path=None):
    path = path or os.environ.get("SEMTSDF_LIB", os.path.join(ROOT, "slam-maskrcnn_amd", "semtsdf", "libsemtsdf.so"))
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def lib_build_key(path=None):
    """The build key compiled into the library (semtsdf_build_key, __graft_entry__.build_key)."""
    import ctypes

    path = path or os.environ.get("SEMTSDF_LIB", os.path.join(ROOT, "slam-maskrcnn_amd", "semtsdf", "libsemtsdf.so"))
    try:
        fn = ctypes.CDLL(path).semtsdf_build_key
    except (OSError, AttributeError):
        return None
    fn.restype = ctypes.c_char_p
    return fn().decode()


def main():
    d, pat, out, dim = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    n_gpus = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/[pe]*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if "FETCH_SIZE" not in agg or "WRITE_SIZE" not in agg:
        raise SystemExit(f"no FETCH_SIZE/WRITE_SIZE rows for {pat!r} under {d}")
    fetch_kib = sum(agg["FETCH_SIZE"]) / len(agg["FETCH_SIZE"])
    write_kib = sum(agg["WRITE_SIZE"]) / len(agg["WRITE_SIZE"])
    fetch = 2.0 * fetch_kib * 1024.0
    write = write_kib * 1024.0
    rec = {"kernel": pat, "dim": dim, "n_gpus": n_gpus, "dispatches": len(agg["FETCH_SIZE"]),
           "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
           "fetch_bytes": fetch, "write_bytes": write, "bytes_per_launch": fetch + write,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE x1", "calibration": CALIBRATION,
           "lib_sha256": lib_sha256(),
           "build_key": lib_build_key()}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
