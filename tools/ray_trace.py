"""Trace the slowest rays of one label render sample by sample (diagnostic, approximate:
float64 numpy, full steps only).  Run with SEMTSDF_RAY_STATS=<file> so the render dumps
its per-pixel march counters; the slowest pixels are then re-marched here against the
downloaded sdf and an 8^3 brick-min map (corners included), printing run lengths of
skippable / evaluated samples and the sdf range of each evaluated run.

    SEMTSDF_RAY_STATS=/tmp/rs.bin python3 tools/ray_trace.py ANGLE [NPIX]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))
import semtsdf  # noqa: E402
from semtsdf import _lib as L  # noqa: E402
from semtsdf.synth import SyntheticStream  # noqa: E402

KI = (520.9, 521.0, 325.1, 249.7)
angle = float(sys.argv[1]) if len(sys.argv) > 1 else 0.3
npick = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rs_path = os.environ["SEMTSDF_RAY_STATS"]
W, H = 640, 480
npx = W * H

st = SyntheticStream(seed=1, noise=True)
f0 = st.frame(0)
p = semtsdf.default_params(512, KI, W, H)
semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
vol = semtsdf.Volume(p, 0)
for k in range(1, 9):
    fr = st.frame(k)
    vol.parse_frame(fr.depth, fr.rgb, np.ascontiguousarray(fr.mask), (fr.w2c @ f0.c2w).astype(np.float32))
dist = float(np.mean(f0.depth[f0.depth > 0]) / 5000.0)
s2w, c = semtsdf.orbit_camera(list(p.Kinv), angle, dist)
if os.path.exists(rs_path):
    os.remove(rs_path)
img = vol.raycast(s2w, c, L.RENDER_LABEL)
raw = np.fromfile(rs_path, dtype=np.uint32)
cnt = raw[:npx * 4].reshape(H, W, 4).astype(np.int64)  # iters, lookups, evals, skipped
sdf = vol.download(sdf=True, wt=False, color=False)["sdf"].reshape(tuple(p.dim))
vol.close()

vx = float(p.voxel[0])
thr = vx / 2.0 * (1.0 + 2.0 ** -16)
start = np.array(p.vol_start[:3], np.float64)
dims = np.array(p.dim[:3])
# brick min over the 8 corners of every sample whose base voxel lies in the brick
m = sdf
for ax in range(3):
    sh = np.concatenate([np.take(m, np.arange(1, m.shape[ax]), axis=ax), np.take(m, [m.shape[ax] - 1], axis=ax)],
                        axis=ax)
    m = np.minimum(m, sh)
nb = dims // 8
bmin = m.reshape(nb[0], 8, nb[1], 8, nb[2], 8).min(axis=(1, 3, 5))
del m
print(f"view {angle}: voxel {vx:.5f} m, thr {thr:.6f}; skippable bricks {np.mean(bmin >= thr):.3f}; "
      f"iters mean {cnt[..., 0].mean():.2f} max {cnt[..., 0].max()}")

S = np.array(s2w, np.float64).reshape(4, 4)
o = np.array(c, np.float64)


def trilinear(i):
    b = np.floor(i)
    f = i - b
    b = b.astype(np.int64)
    x0 = np.clip(b, 0, dims - 1)
    x1 = np.clip(b + 1, 0, dims - 1)
    v = 0.0
    for a in range(2):
        for bb in range(2):
            for cc in range(2):
                w = (f[0] if a else 1 - f[0]) * (f[1] if bb else 1 - f[1]) * (f[2] if cc else 1 - f[2])
                v += w * sdf[(x1 if a else x0)[0], (x1 if bb else x0)[1], (x1 if cc else x0)[2]]
    return v


order = np.argsort(-cnt[..., 0].reshape(-1))
seen = set()
picked = []
for idx in order:
    y, x = divmod(int(idx), W)
    key = (y // 16, x // 16)
    if key in seen:
        continue
    seen.add(key)
    picked.append((y, x))
    if len(picked) == npick:
        break
for (y, x) in picked:
    tgt = S[:3, :3] @ np.array([x, y, 1.0]) + S[:3, 3]
    d = tgt - o
    d /= np.linalg.norm(d)
    with np.errstate(divide="ignore"):
        inv = 1.0 / d
    end = np.array(p.vol_end[:3], np.float64)
    tb, tt = inv * (start - o), inv * (end - o)
    t0 = max(np.max(np.minimum(tb, tt)), 0.01)
    t1 = min(np.min(np.maximum(tb, tt)), 100.0)
    runs = []  # [skip?, n, fmin, fmax, first brick, last brick]
    t = t0
    nsamp = 0
    hit = None
    while t < t1:
        i = (o + t * d - start) / vx
        bi = tuple(np.clip(np.floor(i).astype(np.int64), 0, dims - 1) // 8)
        skip = bmin[bi] >= thr
        f = None if skip else trilinear(i)
        if not runs or runs[-1][0] != skip:
            runs.append([skip, 0, 9.0, -9.0, bi, bi, set()])
        r = runs[-1]
        r[1] += 1
        r[5] = bi
        r[6].add(bi)
        if f is not None:
            r[2] = min(r[2], f)
            r[3] = max(r[3], f)
            if f < 0:
                hit = t
                break
        t += vx
        nsamp += 1
    print(f"\npixel ({x},{y}) tile ({x // 16},{y // 16}): iters {cnt[y, x, 0]} lookups {cnt[y, x, 1]} "
          f"evals {cnt[y, x, 2]} skipped {cnt[y, x, 3]}; dir ({d[0]:+.3f},{d[1]:+.3f},{d[2]:+.3f}); "
          f"{nsamp} full steps, hit {'none' if hit is None else f'{hit:.3f}'}")
    for r in runs:
        if r[0]:
            print(f"   skip {r[1]:4d} samples, {len(r[6]):3d} bricks {r[4]}..{r[5]}")
        else:
            print(f"   EVAL {r[1]:4d} samples, {len(r[6]):3d} bricks {r[4]}..{r[5]}  f in [{r[2]:+.4f}, {r[3]:+.4f}]")
