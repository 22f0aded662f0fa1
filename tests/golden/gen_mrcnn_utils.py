"""Golden vectors of the detector's box arithmetic, made by executing the reference's own
Mask_RCNN/mrcnn/utils.py functions here (run in this container only; its OUTPUT,
tests/golden/mrcnn_utils_golden.npz, is what the tests read).  utils.py imports TensorFlow and
scikit-image at module level, neither installed, so only the pure-NumPy functions the inference
graph restates are taken from the file's text (by name, with the ast module) and executed:
compute_iou, non_max_suppression (utils.py:58-150), apply_box_deltas (:153-174), generate_anchors and
generate_pyramid_anchors (:588-648), norm_boxes and denorm_boxes (:858-889)."""
from __future__ import annotations

import ast
import os

import numpy as np

REF = "/root/reference/Mask_RCNN/mrcnn/utils.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mrcnn_utils_golden.npz")
NAMES = ["compute_iou", "non_max_suppression", "apply_box_deltas", "generate_anchors", "generate_pyramid_anchors",
         "norm_boxes", "denorm_boxes"]


def load():
    tree = ast.parse(open(REF).read())
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in NAMES]
    assert sorted(n.name for n in body) == sorted(NAMES)
    ns = {"np": np}
    exec(compile(ast.Module(body=body, type_ignores=[]), REF, "exec"), ns)
    return ns


def main():
    u = load()
    rng = np.random.default_rng(7)
    out = {}
    # anchors of the COCO inference configuration (1024 x 1024 image) and of a small one
    for tag, S in (("1024", 1024), ("256", 256)):
        strides = [4, 8, 16, 32, 64]
        shapes = np.array([[int(np.ceil(S / s)), int(np.ceil(S / s))] for s in strides])
        a = u["generate_pyramid_anchors"]((32, 64, 128, 256, 512), [0.5, 1, 2], shapes, strides, 1)
        an = u["norm_boxes"](a, (S, S))
        # every 37th anchor and the sums of all of them (the full 1024 table is 2 MB)
        out[f"anchors_{tag}_every37"] = a[::37]
        out[f"anchors_norm_{tag}_every37"] = an[::37]
        out[f"anchors_{tag}_count"] = np.array(a.shape[0])
        out[f"anchors_{tag}_sum"] = a.sum(axis=0)
        out[f"anchors_norm_{tag}_sum"] = an.astype(np.float64).sum(axis=0)
    # box deltas
    boxes = np.sort(rng.uniform(0, 1, (500, 4)).astype(np.float32).reshape(500, 2, 2), axis=1).reshape(500, 4)[:, [0, 2, 1, 3]]
    boxes = boxes[:, [0, 1, 2, 3]]
    deltas = rng.normal(0, 0.3, (500, 4)).astype(np.float32)
    out["delta_boxes"] = boxes
    out["deltas"] = deltas
    out["applied"] = u["apply_box_deltas"](boxes, deltas)
    # denorm of normalized boxes to a 480 x 640 image
    out["denorm_480_640"] = u["denorm_boxes"](np.clip(boxes, 0, 1), (480, 640))
    # NMS cases: random clustered boxes, three thresholds
    for c in range(6):
        n = [20, 200, 1000, 3000, 64, 65][c]
        ctr = rng.uniform(0, 1, (max(n // 10, 1), 2))
        k = rng.integers(0, ctr.shape[0], n)
        cy, cx = ctr[k, 0] + rng.normal(0, 0.02, n), ctr[k, 1] + rng.normal(0, 0.02, n)
        h, w = rng.uniform(0.02, 0.2, n), rng.uniform(0.02, 0.2, n)
        b = np.stack([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], axis=1).astype(np.float32)
        s = rng.uniform(0, 1, n).astype(np.float32)
        out[f"nms{c}_boxes"] = b
        out[f"nms{c}_scores"] = s
        for t in (0.3, 0.5, 0.7):
            out[f"nms{c}_keep_{t}"] = u["non_max_suppression"](b, s, t)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
