"""Mask producer contract: detector masks[H, W, N] -> u8 instance
labels as Mask_RCNN/dmask.py:47-59 mask_detect makes them (mask_process.py:100 calls it
with depth_image=None).  Golden: tests/golden/masks_golden.npz, made by executing dmask.py
itself (tests/golden/gen_masks.py).  CPU: the oracle restatement against the golden; GPU:
semtsdf_masks_to_labels against the golden, bit for bit, and against the oracle on ties,
the area boundary and the detection-count limits."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

CASES = ("n0", "n1", "n8_edges", "n20", "n64")


def golden():
    z = np.load(os.path.join(GOLDEN, "masks_golden.npz"))
    out = {}
    for c in CASES:
        n = int(z[f"{c}_n"])
        packed = z[f"{c}_masks"]
        m = np.unpackbits(packed, axis=2, count=n, bitorder="little").astype(bool)
        out[c] = (m, z[f"{c}_labels"], int(z[f"{c}_kept"]))
    return out


def tie_case(rng, H=96, W=128, n=24):
    """Equal-area detections overlapping one another (rectangles of three sizes)."""
    m = np.zeros((H, W, n), bool)
    sizes = [(20, 30), (30, 20), (25, 24), (10, 60)]  # 600, 600, 600, 600 px
    for i in range(n):
        h, w = sizes[i % len(sizes)]
        y, x = rng.integers(0, H - h), rng.integers(0, W - w)
        m[y:y + h, x:x + w, i] = True
    return m


def test_oracle_matches_dmask_golden(oracle):
    for c, (m, lab, kept) in golden().items():
        got, k = oracle.masks_to_labels(m)
        assert k == kept, c
        np.testing.assert_array_equal(got, lab, err_msg=c)


def test_oracle_tie_rule_is_stable(oracle):
    m = tie_case(np.random.default_rng(3))
    lab, k = oracle.masks_to_labels(m, min_area=0)
    assert k == m.shape[2]
    # every covered pixel goes to the lowest index among the (equal-area) detections covering it
    cov = m.any(axis=2)
    np.testing.assert_array_equal(lab[cov], m.argmax(axis=2)[cov] + 1)
    assert not lab[~cov].any()


@pytest.mark.gpu
def test_gpu_masks_golden():
    from semtsdf.masks import masks_to_labels

    for c, (m, lab, kept) in golden().items():
        got, k = masks_to_labels(m)
        assert k == kept, c
        np.testing.assert_array_equal(got, lab, err_msg=c)


@pytest.mark.gpu
def test_gpu_masks_ties_boundaries_and_limits(oracle):
    from semtsdf import _lib as L
    from semtsdf.masks import masks_to_labels

    rng = np.random.default_rng(11)
    m = tie_case(rng)
    for min_area in (0, 599, 600, 10**6, -1):
        exp, ek = oracle.masks_to_labels(m, min_area=min_area)
        got, k = masks_to_labels(m, min_area=min_area)
        assert k == ek, min_area
        np.testing.assert_array_equal(got, exp, err_msg=str(min_area))
    # odd sizes (npx not a multiple of the workgroup) and the 255-detection maximum label
    for H, W, n in ((7, 13, 3), (33, 65, 255), (480, 640, 100)):
        mm = rng.random((H, W, n)) < (2.0 / max(n, 1))
        exp, ek = oracle.masks_to_labels(mm, min_area=0)
        got, k = masks_to_labels(mm, min_area=0)
        assert k == ek
        np.testing.assert_array_equal(got, exp, err_msg=f"{H}x{W}x{n}")
    with pytest.raises(L.SemTSDFError):
        masks_to_labels(np.zeros((4, 4, 257), bool))
