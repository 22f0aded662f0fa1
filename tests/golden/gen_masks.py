"""Golden vectors of the mask producer contract, made by executing the reference's own
Mask_RCNN/dmask.py here (run in this container only; its OUTPUT, tests/golden/masks_golden.npz,
is what the tests read).  dmask.py is pure NumPy; mask_detect (dmask.py:47-59) is called
with a stand-in model whose detect() returns the case's masks, so filter_tiny_objects,
preserve_small_objs and the i+1 labelling all run as written.  `np.bool` (dmask.py:50,
removed in NumPy 1.24) is shimmed to `bool`.  Areas of the kept detections are distinct
in every case: NumPy's argsort order for equal areas is implementation-defined, the
build's rule for ties (lower detection index first) is tested separately."""
from __future__ import annotations

import importlib.util
import os

import numpy as np

REF = "/root/reference/Mask_RCNN/dmask.py"
OUT = os.path.dirname(os.path.abspath(__file__))
H, W = 480, 640


def load_dmask():
    spec = importlib.util.spec_from_file_location("dmask_ref", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class StandInModel:
    def __init__(self, masks):
        self.masks = masks

    def detect(self, images, verbose=0):
        return [{"masks": self.masks.copy()}]


def ellipse(rng, areas_seen):
    yy, xx = np.mgrid[0:H, 0:W]
    while True:
        cy, cx = rng.uniform(0, H), rng.uniform(0, W)
        ry, rx = rng.uniform(8, 140), rng.uniform(8, 160)
        m = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
        a = int(m.sum())
        if a > 0 and a not in areas_seen:
            areas_seen.add(a)
            return m


def case(rng, n, exact=False):
    seen = set()
    ms = [ellipse(rng, seen) for _ in range(n)]
    if exact:  # the area > 2000 boundary of filter_tiny_objects (dmask.py:42)
        r = np.zeros((H, W), bool)
        r[100:140, 300:350] = True  # 2000 px: dropped
        s = np.zeros((H, W), bool)
        s[200:240, 100:150] = True
        s[240, 100] = True  # 2001 px: kept
        ms += [r, s]
    return np.stack(ms, axis=2) if ms else np.zeros((H, W, 0), bool)


def main():
    np.bool = bool  # dmask.py:50
    dm = load_dmask()
    rng = np.random.default_rng(2024)
    cases = {"n0": case(rng, 0), "n1": case(rng, 1), "n8_edges": case(rng, 6, exact=True),
             "n20": case(rng, 20), "n64": case(rng, 64)}
    rec = {}
    rgb = np.zeros((H, W, 3), np.uint8)
    for name, masks in cases.items():
        lab = dm.mask_detect(StandInModel(masks), rgb)  # reference code (dmask.py:47-59)
        kept = dm.filter_tiny_objects(masks.copy())
        rec[f"{name}_masks"] = np.packbits(masks, axis=2, bitorder="little")
        rec[f"{name}_n"] = np.int64(masks.shape[2])
        rec[f"{name}_labels"] = lab.astype(np.uint8)
        rec[f"{name}_kept"] = np.int64(kept.shape[2])
        print(name, masks.shape[2], "kept", kept.shape[2], "labels", int(lab.max()))
    np.savez_compressed(os.path.join(OUT, "masks_golden.npz"), **rec)


if __name__ == "__main__":
    main()
