"""Z-slab sharding of the volume across GPUs.

The global z axis (camera depth at frame 0) is cut into chunks of `chunk` planes, dealt to
the shards round by round in boustrophedon order: round r holds chunks r n .. r n + n - 1
and shard s owns position s of even rounds and n - 1 - s of odd ones (interleaving balances
the work: near chunks see more of the frustum than far ones; the alternation evens out a
density that drifts along z).  Each shard stores its chunks back to back, each followed by one
halo plane (the first plane of the next chunk), integrated redundantly so that trilinear
samples at a chunk face need no exchange.  Integrate is pointwise, so the gathered owned
planes of all shards equal the single-device volume bit for bit.

This module mirrors `local_planes` / `local_to_global_z` of the C++ layer
(slam-maskrcnn_amd/csrc/semtsdf_api.cpp, semtsdf_kernels.hip) and provides the gather used
by tests and checkpoint export.
"""
from __future__ import annotations

import contextlib
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

    def pos(self, rnd: int, shard: int) -> int:
        """Position of `shard`'s chunk within round `rnd` (chunk_pos of the kernels)."""
        return self.nshards - 1 - shard if rnd & 1 else shard

    def chunks_of(self, shard: int) -> list[int]:
        if self.nshards == 1:
            return [0]
        n = self.nshards
        rounds = (self.nchunks + n - 1) // n
        return [r * n + self.pos(r, shard) for r in range(rounds) if r * n + self.pos(r, shard) < self.nchunks]

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
        pos = np.where(c & 1, self.nshards - 1 - shard, shard)
        return (c * self.nshards + pos) * self.chunk + w

    def owned_local(self, shard: int) -> np.ndarray:
        """Boolean mask over local planes: True for planes this shard owns (not halo)."""
        g = self.local_to_global(shard)
        if self.nshards == 1:
            return np.ones(g.size, bool)
        w = np.arange(g.size) % (self.chunk + 1)
        return (w < self.chunk) & (g < self.dimz)

    def owner(self, z: int) -> int:
        if self.nshards == 1:
            return 0
        c = z // self.chunk
        return self.pos(c // self.nshards, c % self.nshards)

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


# ---------------------------------------------------------------------------------------
# Z-sharded raycast / association protocol (include/semtsdf.h "Z-sharded raycast").
# ---------------------------------------------------------------------------------------
def _exchange_code(exchange: str) -> int:
    from . import _lib as L

    if exchange not in ("allgather", "min"):
        raise ValueError(f"exchange must be 'allgather' or 'min', got {exchange!r}")
    return L.EXCHANGE_MIN if exchange == "min" else L.EXCHANGE_ALLGATHER


def _run_ray_protocol(members, exchange_step, kind, cam, c, stream, exchange: int):
    """members: [Volume] of the shards driven by this process (one per rank in a distributed
    group; all of them for an in-process group).  exchange_step(step) -> (send_ptrs, fn):
    the send buffer of every member for this step and the function that exchanges them
    and returns the device pointer of the exchanged records.  Returns that pointer after
    the last step (the input of render_finish / assoc_partial)."""
    import ctypes as C

    from . import _lib as L

    lib = L.load()
    camv = L.f32(cam, 16)
    cv = L.f32(c, 3) if c is not None else None
    nsteps = C.c_int()
    rec = C.c_size_t()
    for vol in members:
        L.check(lib.semtsdf_shard_ray_begin(vol.handle, int(kind), L.ptr(camv), L.ptr(cv), int(exchange), C.byref(rec),
                                            C.byref(nsteps)))
    gathered = None
    for step in range(nsteps.value):
        sends, fn = exchange_step(step)
        for vol, send in zip(members, sends):
            L.check(lib.semtsdf_shard_ray_step(vol.handle, step, C.c_void_p(gathered) if step else None,
                                               C.c_void_p(send), stream))
        gathered = fn()
    return gathered


class LocalShardGroup:
    """All shards of a Z-sharded volume driven from one process (tests, or several shards
    per GPU): the exchange is device-to-device copies (all-gather) or an element-wise int64
    minimum (the all-reduce MIN) on one stream."""

    def __init__(self, vols, exchange: str = "allgather"):
        from . import _lib as L
        from .volume import DeviceBuffer

        self.vols = list(vols)
        self.n = len(self.vols)
        self.exchange = _exchange_code(exchange)
        v0 = self.vols[0]
        self.W, self.H = v0.W, v0.H
        npx = self.W * self.H
        self.rec = 8 * npx
        self.send = [DeviceBuffer(self.rec) for _ in self.vols]
        self.gathered = DeviceBuffer((self.n if self.exchange == L.EXCHANGE_ALLGATHER else 1) * self.rec)
        self.partial = [DeviceBuffer(8 * L.ASSOC_PARTIAL_LEN) for _ in self.vols]
        self.reduced = DeviceBuffer(8 * L.ASSOC_PARTIAL_LEN)
        self.stream = v0.stream  # every call goes on shard 0's stream: one order for all

    def _s(self):
        import ctypes as C

        return C.c_void_p(self.stream)

    def _exchange(self):
        import ctypes as C

        from . import _lib as L

        lib = L.load()
        if self.exchange == L.EXCHANGE_ALLGATHER:
            for r, sb in enumerate(self.send):
                L.check(lib.semtsdf_memcpy(C.c_void_p(self.gathered.ptr + r * self.rec), C.c_void_p(sb.ptr), self.rec, 3,
                                           self._s()))
        else:
            L.check(lib.semtsdf_memcpy(C.c_void_p(self.gathered.ptr), C.c_void_p(self.send[0].ptr), self.rec, 3,
                                       self._s()))
            for sb in self.send[1:]:
                L.check(lib.semtsdf_min_i64(C.c_void_p(self.gathered.ptr), C.c_void_p(sb.ptr), self.rec // 8,
                                            self._s()))
        return self.gathered.ptr

    def _protocol(self, kind, cam, c):
        sends = [b.ptr for b in self.send]
        return _run_ray_protocol(self.vols, lambda step: (sends, self._exchange), kind, cam, c, self._s(),
                                 self.exchange)

    def raycast_dev(self, s2w, c, mode, out_ptr: int, t_ptr: int | None = None):
        import ctypes as C

        from . import _lib as L

        g = self._protocol(mode, s2w, c)
        # every shard can composite the exchanged records; shard 0 writes the image
        L.check(L.load().semtsdf_shard_render_finish(self.vols[0].handle, C.c_void_p(g), C.c_void_p(out_ptr),
                                                     C.c_void_p(t_ptr) if t_ptr else None, self._s()))

    def raycast(self, s2w, c, mode, want_t=False):
        import numpy as np

        from .volume import DeviceBuffer

        npx = self.W * self.H
        ob = DeviceBuffer(npx * 3)
        tb = DeviceBuffer(npx * 4) if want_t else None
        self.raycast_dev(s2w, c, mode, ob.ptr, tb.ptr if tb else None)
        out = np.zeros((self.H, self.W, 3), np.uint8)
        ob.download(out, self.stream)
        t = None
        if tb:
            t = np.zeros((self.H, self.W), np.float32)
            tb.download(t, self.stream)
        self.vols[0].sync()
        return (out, t) if want_t else out

    def associate_dev(self, mask_ptrs, E, want_stats=False):
        """mask_ptrs: one device mask per shard (identical contents); each is relabelled."""
        import ctypes as C

        from . import _lib as L

        lib = L.load()
        g = self._protocol(L.RAY_ASSOC, E, None)
        for v, m, pb in zip(self.vols, mask_ptrs, self.partial):
            L.check(lib.semtsdf_shard_assoc_partial(v.handle, C.c_void_p(g), C.c_void_p(m), C.c_void_p(pb.ptr),
                                                    self._s()))
        _sum_int64_dev([pb.ptr for pb in self.partial], self.reduced.ptr, L.ASSOC_PARTIAL_LEN, self.stream)
        stats = [L.AssocStats() if want_stats else None for _ in self.vols]
        byref = lambda st: C.byref(st) if st is not None else None
        # every shard certifies the same reduced sums: all decide, or all need the pixels
        rc = lib.semtsdf_shard_assoc_apply(self.vols[0].handle, C.c_void_p(self.reduced.ptr), C.c_void_p(mask_ptrs[0]),
                                           byref(stats[0]), self._s())
        if rc == L.NEED_PIXELS:
            self._apply_exact(g, mask_ptrs, stats)
            return stats
        L.check(rc)
        for v, m, st in zip(self.vols[1:], mask_ptrs[1:], stats[1:]):
            L.check(lib.semtsdf_shard_assoc_apply(v.handle, C.c_void_p(self.reduced.ptr), C.c_void_p(m), byref(st),
                                                  self._s()))
        return stats

    def _apply_exact(self, g, mask_ptrs, stats):
        """The decision's exact path: every shard's per-pixel data, summed (int32), then
        decide + relabel on each shard."""
        import ctypes as C

        from . import _lib as L
        from .volume import DeviceBuffer

        lib = L.load()
        nw = self.W * self.H * L.ASSOC_PIXEL_WORDS
        parts = [DeviceBuffer(4 * nw) for _ in self.vols]
        for v, pb in zip(self.vols, parts):
            L.check(lib.semtsdf_shard_assoc_pixels(v.handle, C.c_void_p(g), C.c_void_p(pb.ptr), self._s()))
        px = DeviceBuffer(4 * nw)
        _sum_int32_dev([pb.ptr for pb in parts], px.ptr, nw, self.stream)
        for v, m, st in zip(self.vols, mask_ptrs, stats):
            L.check(lib.semtsdf_shard_assoc_apply_exact(v.handle, C.c_void_p(self.reduced.ptr), C.c_void_p(px.ptr),
                                                        C.c_void_p(m), C.byref(st) if st is not None else None,
                                                        self._s()))
        self.vols[0].sync()  # the staging buffers are freed on return

    def parse_frame_dev(self, depth_ptr, rgb_ptr, mask_ptrs, E):
        if self.vols[0].state().n_obs > 0:
            self.associate_dev(mask_ptrs, E)
        for v, m in zip(self.vols, mask_ptrs):  # each integrate advances its handle's n_obs (ABI 12)
            v.integrate_dev(depth_ptr, rgb_ptr, m, E, self.stream)


def _sum_int32_dev(ptrs, out_ptr, n, stream):
    """out = sum of the int32 vectors at ptrs (device), via host staging (tests only)."""
    import ctypes as C

    import numpy as np

    from . import _lib as L

    lib = L.load()
    acc = np.zeros(n, np.int32)
    tmp = np.zeros(n, np.int32)
    for p in ptrs:
        L.check(lib.semtsdf_memcpy(L.ptr(tmp), C.c_void_p(p), 4 * n, 2, C.c_void_p(stream)))
        L.check(lib.semtsdf_stream_sync(C.c_void_p(stream)))
        acc += tmp
    L.check(lib.semtsdf_memcpy(C.c_void_p(out_ptr), L.ptr(acc), 4 * n, 1, C.c_void_p(stream)))
    L.check(lib.semtsdf_stream_sync(C.c_void_p(stream)))


def _sum_int64_dev(ptrs, out_ptr, n, stream):
    """out = sum of the int64 vectors at ptrs (device), via host staging (tests only: the
    distributed path uses an all-reduce)."""
    import ctypes as C

    import numpy as np

    from . import _lib as L

    lib = L.load()
    acc = np.zeros(n, np.int64)
    tmp = np.zeros(n, np.int64)
    for p in ptrs:
        L.check(lib.semtsdf_memcpy(L.ptr(tmp), C.c_void_p(p), 8 * n, 2, C.c_void_p(stream)))
        L.check(lib.semtsdf_stream_sync(C.c_void_p(stream)))
        acc += tmp
    L.check(lib.semtsdf_memcpy(C.c_void_p(out_ptr), L.ptr(acc), 8 * n, 1, C.c_void_p(stream)))


class DistShardGroup:
    """One shard per rank of a torch.distributed process group (RCCL on MI355X; gloo for
    CPU-side rehearsal).  Buffers are torch CUDA tensors.  The volume's own HIP stream is
    made torch's current stream (an ExternalStream) around every call, so the library's
    kernels and the collectives (which order themselves after the current stream) share
    one order; torch's default stream would be the NULL stream, which the non-blocking
    volume stream does not synchronise with.

    exchange "min" (default): between protocol steps one all_reduce(MIN) of the 8-byte
    int64 records (2.46 MB per rank at 640x480, whatever the group size; the step buffers
    alternate so a step reads the previous step's reduced records while writing its own);
    "allgather": all_gather_into_tensor of every rank's records (N x 2.46 MB)."""

    def __init__(self, vol, group=None, exchange: str = "min"):
        import torch
        import torch.distributed as dist

        from . import _lib as L

        self.vol = vol
        self.group = group
        self.dist = dist
        self.n = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if vol.params.z_nshards != self.n or vol.params.z_shard != self.rank:
            raise ValueError("volume shard does not match the process group rank")
        self.exchange = _exchange_code(exchange)
        self.W, self.H = vol.W, vol.H
        npx = self.W * self.H
        dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.tstream = torch.cuda.ExternalStream(vol.stream, device=dev)
        self.bufs = [torch.empty(npx, dtype=torch.int64, device=dev) for _ in range(2)]
        self.gathered = torch.empty(self.n * npx, dtype=torch.int64, device=dev) \
            if self.exchange == L.EXCHANGE_ALLGATHER else None
        self.partial = torch.empty(L.ASSOC_PARTIAL_LEN, dtype=torch.int64, device=dev)
        self.nccl = dist.get_backend(group) == "nccl"
        self._parts = None if (self.nccl or self.gathered is None) else list(self.gathered.view(self.n, npx).unbind(0))

    def _stream(self):
        import ctypes as C

        return C.c_void_p(self.vol.stream)

    @contextlib.contextmanager
    def _on_stream(self):
        """Run a call on the volume's stream, ordered both ways against the caller's current
        torch stream: inputs the caller wrote on its stream are ready before the library reads
        them, and the caller's stream waits for the call's outputs (tensors allocated here are
        also recorded as used on the caller's stream)."""
        import torch

        caller = torch.cuda.current_stream(self.device)
        if caller.cuda_stream != self.tstream.cuda_stream:
            self.tstream.wait_stream(caller)
        with torch.cuda.stream(self.tstream):
            yield caller
        if caller.cuda_stream != self.tstream.cuda_stream:
            caller.wait_stream(self.tstream)

    def _exchange_step(self, step):
        from . import _lib as L

        send = self.bufs[step % 2] if self.exchange == L.EXCHANGE_MIN else self.bufs[0]

        def fn():
            if self.exchange == L.EXCHANGE_MIN:
                self.dist.all_reduce(send, op=self.dist.ReduceOp.MIN, group=self.group)
                return send.data_ptr()
            if self.nccl:
                self.dist.all_gather_into_tensor(self.gathered, send, group=self.group)
            else:
                self.dist.all_gather(self._parts, send, group=self.group)
            return self.gathered.data_ptr()

        return [send.data_ptr()], fn

    def raycast_dev(self, s2w, c, mode, out_ptr: int, t_ptr: int | None = None):
        import ctypes as C

        from . import _lib as L

        with self._on_stream():
            g = _run_ray_protocol([self.vol], self._exchange_step, mode, s2w, c, self._stream(), self.exchange)
            L.check(L.load().semtsdf_shard_render_finish(self.vol.handle, C.c_void_p(g), C.c_void_p(out_ptr),
                                                         C.c_void_p(t_ptr) if t_ptr else None, self._stream()))

    def raycast(self, s2w, c, mode, want_t=False):
        import torch

        # allocated on the caller's stream (the caching allocator then keeps them alive for
        # that stream's consumers); the call orders the volume's stream around itself
        out = torch.empty((self.H, self.W, 3), dtype=torch.uint8, device=self.device)
        t = torch.empty((self.H, self.W), dtype=torch.float32, device=self.device) if want_t else None
        self.raycast_dev(s2w, c, mode, out.data_ptr(), t.data_ptr() if t is not None else None)
        return (out, t) if want_t else out

    def associate_dev(self, mask_ptr: int, E, want_stats=False):
        import ctypes as C

        from . import _lib as L

        lib = L.load()
        with self._on_stream():
            g = _run_ray_protocol([self.vol], self._exchange_step, L.RAY_ASSOC, E, None, self._stream(),
                                  self.exchange)
            L.check(lib.semtsdf_shard_assoc_partial(self.vol.handle, C.c_void_p(g), C.c_void_p(mask_ptr),
                                                    C.c_void_p(self.partial.data_ptr()), self._stream()))
            self.dist.all_reduce(self.partial, op=self.dist.ReduceOp.SUM, group=self.group)
            st = L.AssocStats() if want_stats else None
            rc = lib.semtsdf_shard_assoc_apply(self.vol.handle, C.c_void_p(self.partial.data_ptr()),
                                               C.c_void_p(mask_ptr), C.byref(st) if st is not None else None,
                                               self._stream())
            if rc == L.NEED_PIXELS:
                # labels too close to call from the reduced sums (every rank certifies the same
                # sums, so all take this branch): the per-pixel data of every shard, one
                # all-reduce(SUM) over int32 words, then the exact decision
                import torch

                px = torch.empty(self.W * self.H * L.ASSOC_PIXEL_WORDS, dtype=torch.int32, device=self.device)
                L.check(lib.semtsdf_shard_assoc_pixels(self.vol.handle, C.c_void_p(g), C.c_void_p(px.data_ptr()),
                                                       self._stream()))
                self.dist.all_reduce(px, op=self.dist.ReduceOp.SUM, group=self.group)
                L.check(lib.semtsdf_shard_assoc_apply_exact(self.vol.handle, C.c_void_p(self.partial.data_ptr()),
                                                            C.c_void_p(px.data_ptr()), C.c_void_p(mask_ptr),
                                                            C.byref(st) if st is not None else None, self._stream()))
            else:
                L.check(rc)
        return st

    def parse_frame_dev(self, depth_ptr: int, rgb_ptr: int, mask_ptr: int, E, want_stats=False):
        """One frame of the sharded pipeline (association when n_obs > 0, integrate); returns the
        association's stats when want_stats (None without an association)."""
        st = None
        with self._on_stream():
            if self.vol.state().n_obs > 0:
                st = self.associate_dev(mask_ptr, E, want_stats=want_stats)
            self.vol.integrate_dev(depth_ptr, rgb_ptr, mask_ptr, E, self._stream())  # advances n_obs
        return st
