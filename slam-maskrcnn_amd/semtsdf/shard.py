"""Z-slab sharding of the volume across GPUs.

The global z axis (camera depth at frame 0) is cut into chunks of `chunk` planes; chunk c
belongs to shard c % nshards (interleaving balances the work: near chunks see more of the
frustum than far ones).  Each shard stores its chunks back to back, each followed by one
halo plane (the first plane of the next chunk), integrated redundantly so that trilinear
samples at a chunk face need no exchange.  Integrate is pointwise, so the gathered owned
planes of all shards equal the single-device volume bit for bit.

This module mirrors `local_planes` / `local_to_global_z` of the C++ layer
(slam-maskrcnn_amd/csrc/semtsdf_api.cpp, semtsdf_kernels.hip) and provides the gather used
by tests and checkpoint export.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class ShardLayout:
    dimz: int
    nshards: int
    chunk: int

    def __post_init__(self):
        if self.nshards < 1 or self.chunk < 1:
            raise ValueError("nshards and chunk must be >= 1")

    @property
    def halo(self) -> int:
        return 1 if self.nshards > 1 else 0

    @property
    def nchunks(self) -> int:
        return (self.dimz + self.chunk - 1) // self.chunk if self.nshards > 1 else 1

    def chunks_of(self, shard: int) -> list[int]:
        if self.nshards == 1:
            return [0]
        return list(range(shard, self.nchunks, self.nshards))

    def local_planes(self, shard: int) -> int:
        if self.nshards == 1:
            return self.dimz
        return len(self.chunks_of(shard)) * (self.chunk + 1)

    def local_to_global(self, shard: int) -> np.ndarray:
        """Global z of every local plane (may be >= dimz for the last halo plane)."""
        if self.nshards == 1:
            return np.arange(self.dimz)
        per = self.chunk + 1
        l = np.arange(self.local_planes(shard))
        c, w = l // per, l % per
        return (c * self.nshards + shard) * self.chunk + w

    def owned_local(self, shard: int) -> np.ndarray:
        """Boolean mask over local planes: True for planes this shard owns (not halo)."""
        g = self.local_to_global(shard)
        if self.nshards == 1:
            return np.ones(g.size, bool)
        w = np.arange(g.size) % (self.chunk + 1)
        return (w < self.chunk) & (g < self.dimz)

    def owner(self, z: int) -> int:
        return 0 if self.nshards == 1 else (z // self.chunk) % self.nshards

    def gather(self, locals_: list[np.ndarray], dimx: int, dimy: int) -> np.ndarray:
        """Assemble per-shard arrays [dimx, dimy, local_planes(s), ...] into the global
        [dimx, dimy, dimz, ...] array from the owned planes."""
        first = locals_[0]
        extra = first.shape[3:] if first.ndim > 3 else ()
        out = np.zeros((dimx, dimy, self.dimz) + extra, dtype=first.dtype)
        for s, a in enumerate(locals_):
            g = self.local_to_global(s)
            own = self.owned_local(s)
            out[:, :, g[own]] = a[:, :, own]
        return out

    def check_halo(self, locals_: list[np.ndarray]) -> bool:
        """Halo planes equal the owner's plane (redundant integration is identical)."""
        if self.nshards == 1:
            return True
        for s, a in enumerate(locals_):
            g = self.local_to_global(s)
            halo = ~self.owned_local(s) & (g < self.dimz)
            for li in np.nonzero(halo)[0]:
                z = int(g[li])
                o = self.owner(z)
                lo = int(np.nonzero((self.local_to_global(o) == z) & self.owned_local(o))[0][0])
                if not np.array_equal(a[:, :, li], locals_[o][:, :, lo]):
                    return False
        return True
