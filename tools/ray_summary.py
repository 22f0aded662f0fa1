"""Summarise a SEMTSDF_RAY_STATS dump (per-pixel iters, lookups, evals, skipped; per-wave ticks)."""
import sys
import numpy as np
W, H = 640, 480
npx = W * H
raw = np.fromfile(sys.argv[1], dtype=np.uint32)
words = npx * 4 + ((npx + 63) // 64 + 64) * 4
nrec = raw.size // words
r = raw[(nrec - 1) * words:nrec * words]
px = r[:npx * 4].reshape(npx, 4).astype(np.int64)
names = ["iters", "lookups", "evals", "skipped"]
for i, n in enumerate(names):
    v = px[:, i]
    print(f"{n:8s} mean {v.mean():7.2f} p50 {np.percentile(v,50):6.0f} p90 {np.percentile(v,90):6.0f} max {v.max():6d}")
# per wave (16x16 tiles, 4 waves per tile = 4 rows of 16)
tiles = px.reshape(H // 16, 16, W // 16, 16, 4).transpose(0, 2, 1, 3, 4).reshape(-1, 4, 64, 4)
wmax = tiles[..., 0].max(axis=2)
wmean = tiles[..., 0].mean(axis=2)
print("per-wave iters: mean of max %.1f, mean of mean %.1f -> lane efficiency %.2f" % (wmax.mean(), wmean.mean(), wmean.mean() / wmax.mean()))
w = r[npx * 4:].view(np.uint64)[: (npx // 64) * 2].reshape(-1, 2).astype(np.int64)
w = w[w[:, 0] > 0]
d = (w[:, 1] - w[:, 0]) / 100.0  # 100 MHz ticks -> us
print("wave durations us: mean %.1f p50 %.1f p90 %.1f max %.1f; span %.1f us" % (d.mean(), np.percentile(d, 50), np.percentile(d, 90), d.max(), (w[:, 1].max() - w[:, 0].min()) / 100.0))
# slowest waves: their lanes' march counters (wave w of tile t covers rows 4w..4w+3 of the tile)
dur = np.zeros(len(w))
order = np.argsort(-d)[:12]
allw = r[npx * 4:].view(np.uint64)[: (npx // 64) * 2].reshape(-1, 2).astype(np.int64)
valid = np.nonzero(allw[:, 0] > 0)[0]
for i in order:
    wid = valid[i]
    tile, sub = divmod(int(wid), 4)
    ty, tx = divmod(tile, W // 16)
    ys = slice(ty * 16 + sub * 4, ty * 16 + sub * 4 + 4)
    xs = slice(tx * 16, tx * 16 + 16)
    blk = px.reshape(H, W, 4)[ys, xs].reshape(-1, 4)
    print("wave %5d tile (%2d,%2d) %6.1f us  iters max %3d mean %5.1f  lookups max %3d  evals max %3d mean %5.1f  skipped max %3d"
          % (wid, tx, ty, d[i], blk[:, 0].max(), blk[:, 0].mean(), blk[:, 1].max(), blk[:, 2].max(), blk[:, 2].mean(), blk[:, 3].max()))
# distribution of per-lane work in the slowest 5% of waves vs all
