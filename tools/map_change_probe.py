"""Probe (not part of the product): how much of the octant distance map changes per frame of the
bench's C3 stream.  The map refresh after each integrate (dirty-quad plain/dilate + three octant
passes over the whole brick grid, ≈ 37 us of the live frame) could be restricted to the bricks within
the distance cap of the bricks whose skippability changed; this measures that region.
Usage: python tools/map_change_probe.py [FRAMES] [DIM]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    import semtsdf
    from semtsdf import _lib as L
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=1, noise=True)
    frames = [st.frame(k) for k in range(nf)]
    f0 = frames[0]
    from semtsdf.config import TUM_INTRINSICS
    p = semtsdf.default_params(D, TUM_INTRINSICS, f0.depth.shape[1], f0.depth.shape[0])
    semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
    vol = semtsdf.Volume(p, 0)
    nb = D // 8
    prev = None
    cap = 16
    for k, fr in enumerate(frames):
        E = (fr.w2c @ f0.c2w).astype(np.float32)  # bench.py's extrinsic (frame 0 places the volume)
        vol.parse_frame(fr.depth, fr.rgb, fr.mask.copy(), E)
        w = vol.map_words()
        if w is None:
            print("no octant maps")
            return
        w = w.reshape(nb, nb, nb)
        if prev is not None:
            ch = w != prev
            skip_now = (w.view(np.uint8).reshape(nb, nb, nb, 8) > 0).any(-1)
            skip_prev = (prev.view(np.uint8).reshape(nb, nb, nb, 8) > 0).any(-1)
            sk = skip_now != skip_prev
            idx = np.argwhere(sk)
            if len(idx):
                lo, hi = idx.min(0), idx.max(0)
                ext = np.minimum(hi + cap, nb - 1) - np.maximum(lo - cap, 0) + 1
                region = int(np.prod(ext))
            else:
                lo = hi = None
                region = 0
            print(f"frame {k}: map words changed {int(ch.sum())} of {nb ** 3}; bricks whose skippability changed "
                  f"{int(sk.sum())}, bbox {None if lo is None else (lo.tolist(), hi.tolist())}; bbox + cap region "
                  f"{region} bricks ({100.0 * region / nb ** 3:.1f} %)", flush=True)
        prev = w.copy()


if __name__ == "__main__":
    main()
