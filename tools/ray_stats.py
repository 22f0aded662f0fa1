"""Drive one label render of the pipeline bench state and dump march statistics
(SEMTSDF_RAY_STATS instrumentation) for analysis."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))
import semtsdf  # noqa: E402
from semtsdf import _lib as L  # noqa: E402
from semtsdf.synth import SyntheticStream  # noqa: E402

KI = (520.9, 521.0, 325.1, 249.7)
st = SyntheticStream(seed=1, noise=True)
f0 = st.frame(0)
p = semtsdf.default_params(512, KI, 640, 480)
semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
vol = semtsdf.Volume(p, 0)
for k in range(1, 9):
    fr = st.frame(k)
    m = np.ascontiguousarray(fr.mask)
    vol.parse_frame(fr.depth, fr.rgb, m, (fr.w2c @ f0.c2w).astype(np.float32))
dist = float(np.mean(f0.depth[f0.depth > 0]) / 5000.0)
s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.3, dist)
vol.set_instrumentation(events=True)
for _ in range(3):
    img = vol.raycast(s2w, c, L.RENDER_LABEL)
print("render ms", vol.timing().render_ms / max(vol.timing().n_render, 1))
