"""Fixed cost of one integrate launch: the C3 volume (512^3 semantic) integrating a frame it
cannot see (the pose moves it 100 m away from the camera: every voxel far behind the surfaces, every unit culled), so the kernel
time is its launch, LDS table and list set-up alone; beside it the normal C3 frame.
Usage: python tools/empty_launch.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))
import semtsdf  # noqa: E402
from semtsdf import _lib as L  # noqa: E402
from semtsdf.synth import SyntheticStream  # noqa: E402
from semtsdf.volume import DeviceBuffer  # noqa: E402

st = SyntheticStream(seed=1, noise=True)
f0, f1 = st.frame(0), st.frame(1)
p = semtsdf.default_params(512, (520.9, 521.0, 325.1, 249.7), 640, 480)
semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
vol = semtsdf.Volume(p, 0)
npx = 640 * 480
d, r, m = DeviceBuffer(npx * 2), DeviceBuffer(npx * 3), DeviceBuffer(npx)
d.upload(f1.depth)
r.upload(f1.rgb)
m.upload(f1.gt_ids)
E = (f1.w2c @ f0.c2w).astype(np.float32)
E_away = E.copy()
E_away[2, 3] += 100.0  # the volume 100 m further away: every voxel behind the surfaces (culled)
for name, e in (("visible", E), ("empty", E_away), ("visible", E), ("empty", E_away)):
    for _ in range(5):
        vol.integrate_dev(d.ptr, r.ptr, m.ptr, e)
    vol.sync()
    vol.reset_timing()
    vol.set_instrumentation(events=True, count=False)
    for _ in range(20):
        vol.integrate_dev(d.ptr, r.ptr, m.ptr, e)
    vol.sync()
    tm = vol.timing()
    vol.set_instrumentation(events=False, count=True)
    vol.reset_timing()
    vol.integrate_dev(d.ptr, r.ptr, m.ptr, e)
    tc = vol.timing()
    vol.set_instrumentation(events=False, count=False)
    print(f"{name}: kernel {tm.integrate_ms / tm.n_integrate * 1e3:.1f} us, prep {tm.prep_ms / tm.n_prep * 1e3:.1f} us, "
          f"live units {tc.bricks}, touched {tc.touched}", flush=True)
vol.close()
