"""Summarise a SEMTSDF_WAVE_TRACE dump of k_integrate (build: tools/build_variant.sh wtrace
-DSEMTSDF_WAVE_TRACE=1; run: SEMTSDF_LIB=build/var_wtrace.so SEMTSDF_WAVE_TRACE=<file> ...).

Per integrate call: 65536 wave slots x 8 u64 = [entry, table loaded, after free list, after
full-free list, end, smid | block << 32, groups free | full << 20 | general << 40, 0]; wall
clock at 100 MHz (10 ns ticks).  Prints, per call, the spread of the phase boundaries over the
waves (us after the earliest entry) and the per-phase durations.

    python3 tools/wave_trace.py FILE [free-first|full-first] [CALL ...]
"""
import sys

import numpy as np

TICK_US = 0.01
SLOTS, WORDS = 65536, 8


def pct(x, qs=(0, 10, 50, 90, 99, 100)):
    return " ".join(f"p{q}={np.percentile(x, q):7.2f}" for q in qs)


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64)
    calls = raw.reshape(-1, SLOTS, WORDS)
    order = "free-first"
    args = sys.argv[2:]
    if args and args[0] in ("free-first", "full-first"):
        order, args = args[0], args[1:]
    pick = [int(c) for c in args] or range(len(calls))
    for c in pick:
        r = calls[c]
        r = r[r[:, 0] != 0]
        if not len(r):
            continue
        t0 = r[:, 0].min()
        t = (r[:, :5].astype(np.int64) - int(t0)) * TICK_US
        gn = r[:, 6]
        ga, gb, gg = gn & 0xFFFFF, (gn >> 20) & 0xFFFFF, gn >> 40
        gf, gff = (ga, gb) if order == "free-first" else (gb, ga)
        print(f"call {c}: {len(r)} waves, kernel span {t[:, 4].max():.2f} us "
              f"(groups free {gf.sum()} full {gff.sum()} general {gg.sum()})")
        for i, name in enumerate(["entry", "table", "list1 end", "list2 end", "end"]):
            print(f"  {name:9s} {pct(t[:, i])}")
        d1, d2, d_gen = t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 4] - t[:, 3]
        # list 1 / 2: free / full in the unchained build, full / free in the chained one
        d_free = d1 if order == "free-first" else d2
        d_full = d2 if order == "free-first" else d1
        print(f"  dur free  {pct(d_free)}")
        print(f"  dur full  {pct(d_full)}")
        print(f"  dur gen   {pct(d_gen)}")
        with np.errstate(divide="ignore", invalid="ignore"):
            pf = np.where(gf > 0, d_free / np.maximum(gf, 1), np.nan)
            pg = np.where(gg > 0, d_gen / np.maximum(gg, 1), np.nan)
        print(f"  us/group free {np.nanmean(pf):.2f}  general {np.nanmean(pg):.2f}; "
              f"groups/wave free {gf.mean():.1f} general {gg.mean():.1f}")
        blk = (r[:, 5] >> 32).astype(np.int64)
        xcd = blk % 8
        print("  end by XCD (block % 8): " + " ".join(
            f"{x}:{t[xcd == x, 4].mean():.1f}/{t[xcd == x, 4].max():.1f}" for x in range(8)))
        # the 4 waves of a block share a CU; blocks of one CU: smid
        cu = (r[:, 5] & 0xFFFFFFFF).astype(np.int64) + 4096 * xcd
        ucu, inv = np.unique(cu, return_inverse=True)
        cu_end = np.zeros(len(ucu))
        np.maximum.at(cu_end, inv, t[:, 4])
        cu_mean = np.bincount(inv, weights=t[:, 4]) / np.bincount(inv)
        print(f"  per CU ({len(ucu)} CUs): last wave end p0={cu_end.min():.1f} p50={np.median(cu_end):.1f} "
              f"max={cu_end.max():.1f}; mean wave end p0={cu_mean.min():.1f} p50={np.median(cu_mean):.1f} "
              f"max={cu_mean.max():.1f}")
        end = np.sort(t[:, 4])
        n = len(end)
        print("  waves done by: " + " ".join(f"{q}%={end[min(n - 1, int(n * q / 100))]:.1f}"
                                            for q in (25, 50, 75, 90, 95, 99)))
        hwid = (r[:, 7] & 0xFFFFFFFF).astype(np.int64)
        if hwid.any():  # word 7: HW_ID (SIMD bits 5:4): does a wave's age on its SIMD set its pace?
            simd = (hwid >> 4) & 3
            key = cu * 4 + simd
            uk, kinv = np.unique(key, return_inverse=True)
            rank = np.zeros(len(r), np.int64)
            for k in range(len(uk)):
                idx = np.flatnonzero(kinv == k)
                rank[idx[np.argsort(t[idx, 0], kind="stable")]] = np.arange(idx.size)
            dur = t[:, 4] - t[:, 0]
            print(f"  waves per SIMD: {np.bincount(np.bincount(kinv)).nonzero()[0].tolist()}; by age rank on the "
                  "SIMD (0 = entered first): " + " ".join(
                      f"r{q}: n={int((rank == q).sum())} dur={dur[rank == q].mean():.1f} end={t[rank == q, 4].mean():.1f}"
                      for q in range(int(rank.max()) + 1)))
            per_simd_max = np.zeros(len(uk))
            np.maximum.at(per_simd_max, kinv, t[:, 4])
            per_simd_mean = np.bincount(kinv, weights=t[:, 4]) / np.bincount(kinv)
            print(f"  per SIMD: mean end p0={per_simd_mean.min():.1f} p50={np.median(per_simd_mean):.1f} "
                  f"max={per_simd_mean.max():.1f}; spread within a SIMD (max - mean) p50="
                  f"{np.median(per_simd_max - per_simd_mean):.1f} max={np.max(per_simd_max - per_simd_mean):.1f}")


if __name__ == "__main__":
    main()
