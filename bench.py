"""Benchmark of the semantic TSDF hot path on MI355X (BASELINE.json metric:
"Mvoxel-updates/s + frames/s, 512^3 semantic TSDF @ 640x480").

N = 1 (default): configuration C3.  One step = one frame of the integrate
(src/SfM_CUDA/tsdf.cu:18-70 semantics: SDF + gated colour + 32-bin instance histogram; the
frame prepass + unit cull + integrate kernel) over the whole 512^3 volume, inputs resident
in HBM; value = voxels of the volume x frames / wall time of the K timed steps (the
KinectFusion "voxel updates" convention: every voxel is visited per frame, dead units by
the culler).  Extra objects of the same line:
  roofline      the integrate kernel: algorithmic bytes (the reference's types, §8d) per
                launch / its HIP-event duration, against 8 TB/s; traffic = PMC bytes of the
                same kernel binary (stamped by library hash, tools/traffic.py), else null;
  pipeline      §8d frames/s of C3: per frame the host TUM pose path (groundtruth lines ->
                read_traj -> parse_pos), async H2D of depth + RGB + mask from pinned memory
                on a copy stream, association raycast + relabel, integrate and one live
                raycast view, 100 frames after 5 warm-up frames;
  orbit         the live orbit raycast of kernel.cpp:101-107 (angle += 0.01 at the mean
                depth), views/s;
  c2            C2: 256^3 TSDF + colour (NumPy rule: i32 colour, ungated), frames resident,
                Mvoxel-updates/s and upload + integrate frames/s, roofline on 22 N_touch + 5 W H;
  c4_single_gpu C4's 1024^3 semantic volume on one GPU, one step = integrate + one raycast
                view: the base of the N > 1 strong-scaling lines;
  cpu_baseline  the NumPy restatement of tsdf.py:78-120 (+ SfM gate/histogram) on the host.
N > 1 (torch.distributed.run, one process per GPU, RCCL): configuration C4, strong scaling
of the fixed 1024^3 semantic volume: rank r integrates its interleaved Z-slab shard
(no collective) and every step composites one raycast view across the shards (the
DistShardGroup protocol: an RCCL all-reduce MIN of 8-byte per-pixel records between
its steps); value = 1024^3 x K / max-over-ranks wall time.  Rank 0 first runs the same
workload on the whole volume on its GPU (before any shard exists), so the line carries its
own speedup_vs_1gpu; roofline = the slowest rank's algorithmic bytes / its kernel time.
The N = 1 line measures C3 (512^3), so value_N / value_1 is not a speed-up.
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))

METRIC = "Mvoxel-updates/s + frames/s, 512^3 semantic TSDF @ 640x480"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
KI = (520.9, 521.0, 325.1, 249.7)
W, H = 640, 480
NPX = W * H


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- process group
def dist_setup(n_gpus):
    """One process per GPU (torch.distributed.run).  Backend RCCL ("nccl") by default;
    BENCH_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (device = LOCAL_RANK % count)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and n_gpus > 1:
        raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    device = local
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist

        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        device = local % max(ndev, 1) if backend == "gloo" else local
        torch.cuda.set_device(device)
        dist.init_process_group(backend, init_method="env://")
        pg = dist
    return rank, world, device, pg


def _reduce(pg, device, x: float, op) -> float:
    if pg is None:
        return x
    import torch

    on_gpu = pg.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=f"cuda:{device}" if on_gpu else "cpu")
    pg.all_reduce(t, op=op)
    return float(t.item())


def barrier(pg, device):
    if pg is not None:
        import torch

        if pg.get_backend() == "nccl":
            pg.barrier(device_ids=[device])
        else:
            pg.barrier()
        torch.cuda.synchronize()


def max_over_ranks(pg, device, x: float) -> float:
    return x if pg is None else _reduce(pg, device, x, pg.ReduceOp.MAX)


def sum_over_ranks(pg, device, x: float) -> float:
    return x if pg is None else _reduce(pg, device, x, pg.ReduceOp.SUM)


def gather_over_ranks(pg, device, x: float) -> list:
    """Every rank's value of x (an all-reduce SUM of a one-hot vector)."""
    if pg is None:
        return [x]
    import torch

    n, r = pg.get_world_size(), pg.get_rank()
    on_gpu = pg.get_backend() == "nccl"
    t = torch.zeros(n, dtype=torch.float64, device=f"cuda:{device}" if on_gpu else "cpu")
    t[r] = x
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return [float(v) for v in t.cpu()]


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_slab_worker(job):
    """Integrate one x-slab of the volume with the NumPy restatement (1 BLAS thread).
    Returns (voxel-updates, seconds)."""
    frame, p_geo, x0, x_planes = job
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(limits=1)
    except Exception:  # pragma: no cover
        ctx = None
    depth, rgb, mask, E = frame
    D, Dy, Dz, vs, vx, mu = p_geo
    K = np.eye(4, dtype=np.float32)
    K[(0, 1, 0, 1), (0, 1, 2, 2)] = KI
    n = x_planes * Dy * Dz
    sdf = np.full(n, np.float32(mu), np.float32)
    wt = np.zeros(n, np.int32)
    col = np.zeros((n, 3), np.uint8)
    hist = np.zeros((n, 32), np.uint32)
    vs_s = np.array(vs, np.float64)
    vs_s[0] = vs[0] + x0 * vx[0]  # the slab [x0, x0 + x_planes) in a local buffer
    t0 = time.perf_counter()
    O.numpy_integrate(sdf, wt, col, D, vs_s, vx, mu, K, E, depth, rgb, x_range=(0, x_planes),
                      semantic=True, gate=0.99, mask=mask, hist=hist)
    dt = time.perf_counter() - t0
    if ctx is not None:
        ctx.__exit__(None, None, None)
    return n, dt


def cpu_baseline(frames, p, f0, x_planes=64, slabs=10, workers=1):
    """NumPy restatement of tsdf.py:78-120 (+ SfM gate/histogram) over a bounded sample of
    the 512^3 workload: `slabs` x-slabs of `x_planes` planes around the volume centre, one
    frame each.  workers=1: one core, time = sum of the slab times.  workers>1: x-slab
    multiprocessing (fork; the children only run NumPy), time = wall time of the pool."""
    D, Dy, Dz = p.dim[0], p.dim[1], p.dim[2]
    assert D == Dy == Dz, "the CPU baseline runs on the cubic N=1 volume"
    geo = (D, Dy, Dz, tuple(p.vol_start[:]), tuple(float(v) for v in p.voxel[:]), float(p.mu))
    jobs = []
    for s in range(slabs):
        fr = frames[s % len(frames)]
        E = (fr.w2c @ f0.c2w).astype(np.float64)
        x0 = (D // 2 - x_planes // 2 + (s - slabs // 2) * x_planes) % max(D - x_planes, 1)
        jobs.append(((fr.depth, fr.rgb, fr.mask, E), geo, x0, x_planes))
    if workers <= 1:
        res = [_cpu_slab_worker(j) for j in jobs]
        total = sum(r[0] for r in res)
        t = sum(r[1] for r in res)
    else:
        import multiprocessing as mp

        with mp.get_context("fork").Pool(workers) as pool:
            t0 = time.perf_counter()
            res = pool.map(_cpu_slab_worker, jobs, chunksize=1)
            t = time.perf_counter() - t0
        total = sum(r[0] for r in res)
    return {"value": total / t / 1e6, "unit": "Mvoxel-updates/s", "cores": int(workers), "kind": "port",
            "sample": f"{slabs} x-slabs of {x_planes} planes of the {D}^3 volume, one synthetic frame each "
                      f"({total} voxel-updates, {t:.1f} s{' wall' if workers > 1 else ''}), NumPy restatement of "
                      f"tsdf.py:78-120 + SfM gate/histogram, 1 BLAS thread per "
                      f"{'worker' if workers > 1 else 'process'}"}


def host_cores() -> int:
    """Cores this job may use on the host (the GPU box caps the share via OMP_NUM_THREADS)."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:  # pragma: no cover
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit():
        n = min(n, int(cap))
    return max(1, n)


# ----------------------------------------------------------------------------- helpers
def copy_bandwidth(device: int, nbytes: int = 1 << 30) -> float:
    """Achievable HBM bandwidth (GB/s, read + write) of a float4 device copy (library kernel),
    for context beside the 8 TB/s spec peak."""
    import ctypes as C

    from semtsdf import _lib as L

    out = C.c_double()
    L.check(L.load().semtsdf_copy_bandwidth(int(device), int(nbytes), 5, C.byref(out)))
    return out.value


def loaded_lib_sha256() -> str:
    from semtsdf import _lib as L

    path = os.environ.get("SEMTSDF_LIB", L.LIB_PATH)
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def loaded_build_key() -> str | None:
    """Key of the sources, flags and compiler the loaded library was built from: a driver-side
    rebuild of the same sources keeps it (the .so bytes may differ)."""
    from semtsdf import _lib as L

    lib = L.load()
    if not hasattr(lib, "semtsdf_build_key"):
        return None
    k = lib.semtsdf_build_key()
    k = k.decode() if k else None
    return None if k in (None, "unknown") else k


CALIBRATION = "profiles/r06/calib/calibration.json"  # tools/calib_pmc.sh


def read_traffic(path, dim, world):
    """PMC bytes per launch of the integrate kernel, only if measured on this very library
    build (tools/traffic.py stamps the build key and the binary's SHA-256) and configuration."""
    if not path or not os.path.exists(path):
        return None, "no traffic record"
    try:
        with open(path) as f:
            tj = json.load(f)
    except Exception as e:  # pragma: no cover
        return None, f"unreadable traffic record: {e}"
    if tj.get("dim") != dim or tj.get("n_gpus", 1) != world:
        return None, "traffic record is for another configuration"
    key = loaded_build_key()
    # the x2 / x1 corrections checked on known byte counts of the integrate's access patterns
    cal = f"; corrections calibrated in {CALIBRATION}" if os.path.exists(os.path.join(ROOT, CALIBRATION)) else ""
    if tj.get("build_key") and key == tj["build_key"]:
        return tj.get("bytes_per_launch"), f"PMC FETCH_SIZE x2 + WRITE_SIZE of build key {key[:12]}{cal}"
    if tj.get("lib_sha256") != loaded_lib_sha256():
        return None, "traffic record was measured on another library build"
    return tj.get("bytes_per_launch"), f"PMC FETCH_SIZE x2 + WRITE_SIZE of lib {tj['lib_sha256'][:12]}{cal}"


def place(semtsdf, L, D, f0, dimz=None):
    p = semtsdf.default_params(D, KI, W, H)
    if dimz is not None:
        p.dim[2] = dimz
    semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
    return p


def resident_frames(frames, with_mask=True, ids=False):
    """Depth, RGB and masks of `frames` in HBM (library allocations)."""
    from semtsdf.volume import DeviceBuffer

    n = len(frames)
    dbuf, rbuf = DeviceBuffer(n * NPX * 2), DeviceBuffer(n * NPX * 3)
    mbuf = DeviceBuffer(n * NPX) if with_mask else None
    for i, fr in enumerate(frames):
        dbuf.upload(fr.depth, None, i * NPX * 2)
        rbuf.upload(fr.rgb, None, i * NPX * 3)
        if with_mask:
            mbuf.upload(fr.gt_ids if ids else fr.mask, None, i * NPX)
    return dbuf, rbuf, mbuf


def timed_integrate(vol, step, K, warmup, pg=None, device=0, finish=None):
    """Wall time of K steps (barrier + sync on both sides; `finish`, if given, runs once
    after them inside the timed region), then the same K steps again with kernel events
    (integrate kernel, prepass) and once more counting voxels."""
    for k in range(warmup):
        step(k)
    if finish is not None:
        finish()
    vol.sync()
    barrier(pg, device)
    vol.sync()
    t0 = time.perf_counter()
    for k in range(K):
        step(warmup + k)
    if finish is not None:
        finish()
    vol.sync()
    barrier(pg, device)
    elapsed = time.perf_counter() - t0
    vol.reset_timing()
    vol.set_instrumentation(events=True, count=False)
    for k in range(K):
        step(warmup + k)
    vol.sync()
    tm = vol.timing()
    vol.reset_timing()
    vol.set_instrumentation(events=False, count=True)
    for k in range(K):
        step(warmup + k)
    tc = vol.timing()
    vol.set_instrumentation(events=False, count=False)
    return elapsed, tm, tc


# ----------------------------------------------------------------------------- C3 pipeline
class HipEvent:
    """A HIP event for ordering this process's streams on one device (the upload ring): no
    timing and no system-scope fence (hipEventDisableSystemFence: the consumers are kernels of
    the same device), unlike torch.cuda.Event.  The HIP runtime is torch's (semtsdf._lib loads
    the library after torch, so both resolve libamdhip64.so.7 to the same copy)."""
    _hip = None

    def __init__(self):
        if HipEvent._hip is None:
            h = ctypes.CDLL("libamdhip64.so.7")
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            h.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
            h.hipEventDestroy.argtypes = [ctypes.c_void_p]
            HipEvent._hip = h
        self.ev = ctypes.c_void_p()
        rc = HipEvent._hip.hipEventCreateWithFlags(ctypes.byref(self.ev), 0x2 | 0x20000000)
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags: {rc}")

    @property
    def cuda_event(self):
        return self.ev.value

    def record(self, stream):
        rc = HipEvent._hip.hipEventRecord(self.ev, ctypes.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord: {rc}")

    def __del__(self):
        if HipEvent._hip is not None and self.ev:
            HipEvent._hip.hipEventDestroy(self.ev)

    def wait_on(self, stream):
        rc = HipEvent._hip.hipStreamWaitEvent(ctypes.c_void_p(stream.cuda_stream), self.ev, 0)
        if rc != 0:
            raise RuntimeError(f"hipStreamWaitEvent: {rc}")


def run_pipeline(semtsdf, L, p, local, n_frames=100, n_warm=5):
    """§8d frames/s of C3: host pose path + async H2D (pinned, copy stream) + association
    raycast + relabel + integrate + one live raycast view per frame, in the volume stream's
    order (the reported rate).  "overlapped": the live view of frame k on a render stream
    beside the association of frame k+1 (both only read the volume; frame k+1's integrate
    waits for the view, semtsdf_parse_frame_dev_after) — measured slower: two latency-bound
    marches sharing the CUs stretch each other's tails."""
    import torch

    from semtsdf import pose as P
    from semtsdf import tum
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=1, noise=True)
    n_all = n_frames + n_warm + 1
    t_gen = time.perf_counter()
    frames = [st.frame(k) for k in range(n_all)]
    log(f"[bench] pipeline: generated {n_all} frames in {time.perf_counter() - t_gen:.1f}s")
    with tempfile.TemporaryDirectory() as d:
        gt = os.path.join(d, "groundtruth.txt")
        with open(gt, "w") as f:
            f.write("\n".join(st.tum_lines(n_all)) + "\n")
        traj = tum.read_traj(gt)  # tsdf_utils.py:23-29
    dev = torch.device("cuda", local)
    # pinned host frames (a capture pipeline's buffers): depth u16, rgb u8x3, mask u8 of a
    # frame back to back, copied by one kernel (semtsdf_memcpy kind 4: the runtime's DMA copy
    # from pinned memory blocked the host loop for the transfer, tools/host_overhead.py)
    h_all = torch.empty((n_all, NPX * 6), dtype=torch.uint8).pin_memory()
    for k, fr in enumerate(frames):
        h_all[k, :NPX * 2].copy_(torch.from_numpy(fr.depth.reshape(-1).view(np.uint8)))
        h_all[k, NPX * 2:NPX * 5].copy_(torch.from_numpy(fr.rgb.reshape(-1)))
        h_all[k, NPX * 5:].copy_(torch.from_numpy(fr.mask.reshape(-1)))
    lib = L.load()
    mean_m = tum.mean_depth_m(frames[0].depth)
    ext0_inv = np.linalg.inv(P.parse_pos(traj[0, 1:]))  # frame 0 places the volume (tsdf.cu:173-214)

    def run(overlap, instr=False, fused=False, force_exact=False):
        vol = semtsdf.Volume(p, local)
        if force_exact:  # every association row decided from its exact f32 pixel-order sums
            vol.set_instrumentation(events=False, force_exact=True)
        vstream = torch.cuda.ExternalStream(vol.stream, device=dev)
        cstream = torch.cuda.Stream(device=dev)
        rstream = torch.cuda.Stream(device=dev) if overlap else vstream
        # frame k + ring - lag is uploaded after frame k into the slot frame k - lag used
        ring, lag = 4, 2
        d_all = torch.empty((ring, NPX * 6), dtype=torch.uint8, device=dev)
        slot = [(d_all[s].data_ptr(), d_all[s].data_ptr() + NPX * 2, d_all[s].data_ptr() + NPX * 5)
                for s in range(ring)]
        outs = [torch.empty(NPX * 3, dtype=torch.uint8, device=dev) for _ in range(2)]
        hip_ev = os.environ.get("BENCH_HIP_EVENTS", "1") != "0"
        mk = HipEvent if hip_ev else torch.cuda.Event
        copied = [mk() for _ in range(ring)]
        used = [mk() for _ in range(ring)]
        integrated = mk()
        rendered = mk()

        def wait(stream, ev):
            if hip_ev:
                ev.wait_on(stream)
            else:
                stream.wait_event(ev)
        torch.cuda.synchronize()

        def upload(k):
            s = k % ring
            wait(cstream, used[s])
            L.check(lib.semtsdf_memcpy(ctypes.c_void_p(slot[s][0]), ctypes.c_void_p(h_all[k].data_ptr()), NPX * 6, 4,
                                       ctypes.c_void_p(cstream.cuda_stream)))
            copied[s].record(cstream)

        def frame(k, first):
            s = k % ring
            E = P.relative_pose(P.parse_pos(traj[k, 1:]), ext0_inv)  # host pose path (tsdf.cu:217)
            wait(vstream, copied[s])
            after = rendered.cuda_event if (overlap and not first) else None
            pd, pr, pm = slot[s]
            if fused:  # the view shown after frame k - 1, in the launch of frame k's association
                s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * (k - 1), mean_m)
                vol.parse_frame_view_dev(pd, pr, pm, E, s2w, c, L.RENDER_LABEL, outs[(k - 1) % 2].data_ptr())
                used[s].record(vstream)
                if k + ring - lag < n_all:
                    upload(k + ring - lag)
                return
            vol.parse_frame_dev(pd, pr, pm, E, integrate_after_event=after)
            used[s].record(vstream)
            s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * k, mean_m)
            if overlap:
                integrated.record(vstream)
                wait(rstream, integrated)
            vol.raycast_dev(s2w, c, L.RENDER_LABEL, outs[k % 2].data_ptr(), stream=rstream.cuda_stream)
            if overlap:
                rendered.record(rstream)
            if k + ring - lag < n_all:
                upload(k + ring - lag)

        for k in range(ring - lag):
            upload(1 + k)
        for k in range(1, 1 + n_warm):
            frame(k, k == 1)
        vol.sync()
        torch.cuda.synchronize()
        # the timed frames carry no timing events (each event pair adds a barrier on the stream)
        if instr:  # per-kernel breakdown run: timing events around the kernels
            vol.reset_timing()
            vol.set_instrumentation(events=True, count=False)
        t0 = time.perf_counter()
        for k in range(1 + n_warm, n_all):
            frame(k, False)
        vol.sync()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        tm = vol.timing()
        if fused:  # the view of the last frame (rendered by the next frame's call), untimed
            s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * (n_all - 1), mean_m)
            vol.raycast_dev(s2w, c, L.RENDER_LABEL, outs[(n_all - 1) % 2].data_ptr())
            vol.sync()
        return vol, t1 - t0, tm, outs[(n_all - 1) % 2].clone(), int(vol.state().num_objs)


    vol_s, t_ser, _, img_s, objs_s = run(False)  # serial order: no timing events
    ref_img = img_s.cpu()
    vol_s.close()
    # the reported rate: each frame's call renders the view of the previous frame's state in the
    # launch of its association march (semtsdf_parse_frame_view_dev); same frames, same views
    vol_f, t_fus, tm_f, img_f, objs_f = run(False, fused=True)
    vol_f.close()
    same_f = bool(torch.equal(img_f.cpu(), ref_img)) and objs_f == objs_s
    # the cost of the decision's exact path: the same fused frames with every row forced onto it
    vol_x, t_exact, tm_x, img_x, objs_x = run(False, fused=True, force_exact=True)
    vol_x.close()
    same_x = bool(torch.equal(img_x.cpu(), ref_img)) and objs_x == objs_s
    vol_b, _, tm, _, _ = run(False, instr=True)  # the same frames again, with events
    vol_b.close()
    vol, t_ovl, _, img_o, objs_o = run(True)
    same = bool(torch.equal(img_o.cpu(), ref_img)) and objs_o == objs_s
    # live orbit (kernel.cpp:101-107): angle += 0.01 per view, distance = mean depth
    out = torch.empty(NPX * 3, dtype=torch.uint8, device=dev)
    n_views = 60
    vol.sync()
    tv0 = time.perf_counter()
    for v in range(n_views):
        s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * (v + 1), mean_m)
        vol.raycast_dev(s2w, c, L.RENDER_LABEL, out.data_ptr())
    vol.sync()
    tv1 = time.perf_counter()
    vol.reset_timing()  # kernel time per view: the same views again, with events
    vol.set_instrumentation(events=True, count=False)
    for v in range(n_views):
        s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * (v + 1), mean_m)
        vol.raycast_dev(s2w, c, L.RENDER_LABEL, out.data_ptr())
    vol.sync()
    tr = vol.timing()
    vol.set_instrumentation(events=False, count=False)
    vol.close()
    return {
        "frames_per_s": n_frames / t_fus,
        "ms_per_frame": t_fus * 1e3 / n_frames,
        "serial_frames_per_s": n_frames / t_ser,
        "serial_ms_per_frame": t_ser * 1e3 / n_frames,
        "fused_equals_serial": same_f,
        "view_lag_frames": 1,
        "assoc_decisions": int(tm_f.n_assoc),
        "assoc_exact_frames": int(tm_f.assoc_exact_frames),
        "assoc_exact_rows": int(tm_f.assoc_exact_rows),
        "assoc_pos_max": round(float(tm_f.assoc_pos_max), 6),
        "assoc_exact_note": "decisions (warm-up included) whose certificate left rows to the exact f32 "
                            "pixel-order path (DESIGN.md §4); all_exact_frames_per_s: every row forced onto it",
        "all_exact_frames_per_s": n_frames / t_exact,
        "all_exact_equals_serial": same_x,
        "overlapped_frames_per_s": n_frames / t_ovl,
        "overlapped_equals_serial": same,
        "frames": n_frames, "warmup_frames": n_warm,
        "per_frame": "host TUM pose (read_traj -> parse_pos) + H2D of depth/RGB/mask from pinned memory by a copy kernel on a copy stream "
                     "+ association raycast + relabel + integrate + 1 label raycast view; frames_per_s: the view "
                     "of the state after frame k-1 is rendered in the launch of frame k's association march "
                     "(semtsdf_parse_frame_view_dev: the view a viewer shows after frame k-1, one frame later); "
                     "serial_frames_per_s: view k rendered after frame k's integrate",
        "breakdown_source": "a second serial run of the same frames with timing events around the kernels "
                            "(each event pair adds a barrier; the timed runs carry none)",
        "assoc_ms_per_frame": tm.assoc_ms / max(tm.n_assoc, 1),
        "integrate_ms_per_frame": tm.integrate_ms / max(tm.n_integrate, 1),
        "prep_ms_per_frame": tm.prep_ms / max(tm.n_prep, 1),
        "render_ms_per_view": tm.render_ms / max(tm.n_render, 1),
        "num_objs": objs_s,
    }, {
        "views_per_s": n_views / (tv1 - tv0),
        "render_ms_per_view": tr.render_ms / max(tr.n_render, 1),
        "views": n_views,
        "camera": "viewer.cu:137-146 orbit, angle += 0.01 per view (kernel.cpp:104), dist = mean depth of frame 0",
    }


# ----------------------------------------------------------------------------- mask producer
def run_mask_overlap(semtsdf, L, p, local, frames, f0, n_frames=32, n_warm=3):
    """§8f rank 1 / config C5: the Mask R-CNN producer (semtsdf/maskrcnn.py: the reference's
    ResNet-101-FPN inference graph, mrcnn/model.py, seeded random weights, fp16 MIOpen convolutions, HIP
    NMS) on each frame's RGB in HBM, its masks[H, W, 100] into semtsdf_masks_to_labels (dmask.py rule) on
    a producer stream, feeding parse_frame_dev (association + relabel + integrate) on the volume's
    stream.  "serial": producer and fusion in one stream order; "overlapped": the producer of frame k+1
    on its own stream while frame k fuses (2 label slots, events both ways).  Random weights give
    arbitrary masks, so the volume runs with SEMTSDF_F_ID_SATURATE (ids stop at 32)."""
    import torch

    from semtsdf import maskrcnn as MR
    from semtsdf.masks import masks_to_labels_dev

    dev = torch.device("cuda", local)
    F_ = len(frames)
    rgb = [torch.from_numpy(fr.rgb).to(dev) for fr in frames]
    # fp16 convolutions: 10.1 against 11.5 ms per detect in bf16 (profiles/r06/det/dtype_probe.txt), and
    # closer to the reference's f32 graph (10 mantissa bits against 7); the calibration keeps every
    # layer's output near unit scale, far inside fp16's range
    cfg = MR.Config(DTYPE=torch.float16)
    model = MR.MaskRCNN(cfg, seed=0).to(dev).to(cfg.DTYPE).eval()
    model.calibrate(dev, rgb[0])
    # the whole detect() as one HIP graph replay per frame (falls back to eager launches if the capture
    # is refused)
    try:
        gdet = MR.GraphDetector(model, rgb[0].shape, dev)
        detect = gdet
        graph_note = "HIP graph (torch.cuda.CUDAGraph) of detect(compact=False), one replay per frame"
    except Exception as e:  # pragma: no cover
        detect = lambda im: model.detect(im, compact=False)  # noqa: E731
        graph_note = f"eager launches (graph capture refused: {e!r})"
    ND = cfg.DETECTION_MAX_INSTANCES
    labels = torch.empty((2, NPX), dtype=torch.uint8, device=dev)
    dbuf, rbuf, _ = resident_frames(frames, with_mask=False)
    Es = [(fr.w2c @ f0.c2w).astype(np.float32) for fr in frames]
    pstream = torch.cuda.Stream(device=dev)
    saved_flags = p.flags
    p.flags = saved_flags | L.F_ID_SATURATE
    held = [None, None]  # each slot's detector outputs stay alive until its labels are made

    def run(mode):
        vol = semtsdf.Volume(p, local)
        vstream = torch.cuda.ExternalStream(vol.stream, device=dev)
        ready = [torch.cuda.Event() for _ in range(2)]
        used = [torch.cuda.Event() for _ in range(2)]
        ps = vstream if mode == "serial" else pstream

        def produce(k):
            s = k % 2
            with torch.cuda.stream(ps):
                ps.wait_event(used[s])
                out = detect(rgb[k % F_])
                masks_to_labels_dev(out["masks"].data_ptr(), W, H, ND, labels[s].data_ptr(), stream=ps.cuda_stream)
                held[s] = out
                ready[s].record(ps)

        def fuse(k):
            s, i = k % 2, k % F_
            vstream.wait_event(ready[s])
            vol.parse_frame_dev(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, labels[s].data_ptr(), Es[i])
            used[s].record(vstream)

        def frames_(k0, k1):
            if mode == "serial":
                for k in range(k0, k1):
                    produce(k)
                    fuse(k)
            else:
                produce(k0)
                for k in range(k0, k1):
                    if k + 1 < k1:
                        produce(k + 1)
                    fuse(k)

        frames_(0, n_warm)
        vol.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        frames_(n_warm, n_warm + n_frames)
        vol.sync()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        objs = int(vol.state().num_objs)
        vol.close()
        return dt, objs

    def producer_only(n):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dets = 0
        with torch.cuda.stream(pstream):
            ev0.record(pstream)
            for k in range(n):
                out = detect(rgb[k % F_])
                masks_to_labels_dev(out["masks"].data_ptr(), W, H, ND, labels[k % 2].data_ptr(),
                                    stream=pstream.cuda_stream)
                held[k % 2] = out
            ev1.record(pstream)
        ev1.synchronize()
        for k in range(min(n, F_)):
            dets += int((model.detect(rgb[k], compact=False)["class_ids"] > 0).sum().item())
        return ev0.elapsed_time(ev1) / n, dets / min(n, F_)

    try:
        producer_only(2)
        t_ser, objs_ser = run("serial")
        t_ovl, objs_ovl = run("overlapped")
        prod_ms, dets = producer_only(n_frames)
    finally:
        p.flags = saved_flags
        for b in (dbuf, rbuf):
            b.free()
    return {
        "serial_frames_per_s": round(n_frames / t_ser, 2),
        "overlapped_frames_per_s": round(n_frames / t_ovl, 2),
        "producer_ms_per_frame": round(prod_ms, 4),
        "detections_per_frame": round(dets, 2), "frames": n_frames,
        "num_objs_serial": objs_ser, "num_objs_overlapped": objs_ovl,
        "launch": graph_note,
        "producer": ("Mask R-CNN inference graph of the reference (mrcnn/model.py: ResNet-101-FPN, RPN 6000 -> "
                     "1000 proposals, 81-class heads, 1024x1024 input) in PyTorch-ROCm, fp16 MIOpen convolutions, "
                     "HIP NMS (libsemtsdf_det.so), seeded random weights (no COCO checkpoint offline): detect() -> "
                     "masks[H,W,100] -> semtsdf_masks_to_labels (dmask.py:47-59 rule); volume with "
                     "SEMTSDF_F_ID_SATURATE"),
    }


# ----------------------------------------------------------------------------- C2
def run_c2(semtsdf, L, local, frames, f0, K=30, warmup=3, traffic_json=None, async_prepass=True):
    """C2: 256^3 TSDF + colour (NumPy rule: int32 colour, no gate), synthetic stream."""
    D = 256
    p = place(semtsdf, L, D, f0)
    p.flags = L.F_COLOR_I32
    vol = semtsdf.Volume(p, local)
    dbuf, rbuf, _ = resident_frames(frames, with_mask=False)
    Es = [(fr.w2c @ f0.c2w).astype(np.float32) for fr in frames]

    def step(k):
        i = k % len(frames)
        if async_prepass:  # as the C3 step: the prepass beside the previous frame's integrate
            vol.integrate_dev_async(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, None, Es[i])
        else:
            vol.integrate_dev(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, None, Es[i])

    elapsed, tm, tc = timed_integrate(vol, step, K, warmup)
    kern_ms = tm.integrate_ms / max(tm.n_integrate, 1)
    touched = tc.touched / K
    b = 22.0 * touched + 5.0 * NPX
    # upload + integrate (§8d C2 frames/s): host frames through the library's H2D path
    vol.reset()
    t0 = time.perf_counter()
    for k in range(K):
        fr = frames[k % len(frames)]
        vol.integrate(fr.depth, fr.rgb, None, Es[k % len(frames)])
    vol.sync()
    t_up = time.perf_counter() - t0
    vol.close()
    dbuf.free()
    rbuf.free()
    c2_traffic, c2_src = read_traffic(traffic_json, D, 1)
    # line-granular floor of the state traffic: every 128-B line holding a touched voxel is read
    # and written whole in each of the three state arrays (sdf, weight, colour u8x4), plus the
    # 8-B pixel records read once
    lines = tc.touched_lines / K
    floor = 128.0 * 6 * lines + 8.0 * NPX
    return {
        "workload": "C2: 256^3 TSDF + colour (sdf f32, weight i32, colour i32x3, NumPy rule: colour ungated), "
                    "synthetic 640x480 stream, ground-truth poses",
        "value": round(D ** 3 * K / elapsed / 1e6, 2), "unit": "Mvoxel-updates/s",
        "ms_per_step": round(elapsed * 1e3 / K, 4),
        "integrate_kernel_ms": round(kern_ms, 4),
        "frames_per_s_upload_integrate": round(K / t_up, 1),
        "prepass": "beside the previous integrate (semtsdf_integrate_dev_async)" if async_prepass else "in front",
        "touched_per_frame": int(touched),
        "live_units_per_frame": int(tc.bricks / K),
        "roofline": {"bound": "hbm", "achieved": round(b / (kern_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(b / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": c2_traffic, "traffic_source": c2_src,
                     "algorithmic_bytes_per_launch": int(b), "bytes_rule": "22 N_touch + 5 W H (SURVEY §8d)"},
        "touched_mvox_per_s": round(touched / (kern_ms * 1e-3) / 1e6, 1),
        "touched_lines_per_frame": int(lines),
        "line_floor_bytes_per_launch": int(floor),
        "line_floor_rule": "128 B x 3 arrays (sdf, weight, colour u8x4) x read+write per 128-B sdf line holding a "
                           "touched voxel (tiles of 8 y x 4 z voxels) + 8 B pixel record per pixel",
        "traffic_over_line_floor": round(c2_traffic / floor, 3) if c2_traffic else None,
    }


# ----------------------------------------------------------------------------- C4
def c4_params(semtsdf, L, f0, world=1, rank=0, chunk=64):
    p = place(semtsdf, L, 1024, f0)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
    if world > 1:
        p.z_nshards, p.z_shard, p.z_chunk = world, rank, chunk
    return p


C4_SPEC = ("C4: 1024^3 semantic TSDF (sdf f32, weight i32, colour u8x3, 32-bin u32 histogram); per step one frame "
           "integrated, and after the K steps one label raycast view (the north star's final raycast composite)")


def run_c4_single(semtsdf, L, local, frames, f0, K, warmup, async_prepass=True):
    """C4's 1024^3 semantic volume whole on one GPU (the base of the strong-scaling lines):
    K integrated frames + the final label raycast, then the per-frame variant (integrate +
    one raycast view every step)."""
    from semtsdf.volume import DeviceBuffer

    p = c4_params(semtsdf, L, f0)
    vol = semtsdf.Volume(p, local)
    dbuf, rbuf, mbuf = resident_frames(frames, ids=True)
    Es = [(fr.w2c @ f0.c2w).astype(np.float32) for fr in frames]
    mean_m = float(np.mean(f0.depth[f0.depth > 0]) / 5000.0)
    out = DeviceBuffer(NPX * 3)

    def integ(k):
        i = k % len(frames)
        if async_prepass:  # as the C3 step: the prepass beside the previous frame's integrate
            vol.integrate_dev_async(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, mbuf.ptr + i * NPX, Es[i])
        else:
            vol.integrate_dev(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, mbuf.ptr + i * NPX, Es[i])

    def view(k=0):
        s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * k, mean_m)
        vol.raycast_dev(s2w, c, L.RENDER_LABEL, out.ptr)

    elapsed, tm, tc = timed_integrate(vol, integ, K, warmup, finish=view)
    vol.reset_timing()
    vol.set_instrumentation(events=True, count=False)
    view()
    vol.sync()
    render_ms = vol.timing().render_ms
    vol.set_instrumentation(events=False, count=False)
    Kf = max(4, K // 3)
    elapsed_f, _, _ = timed_integrate(vol, lambda k: (integ(k), view(k)), Kf, 1)
    # the semantic frame: association raycast + relabel of the frame's own (permuted) labels,
    # then the integrate; the masks are relabelled in place, so each step copies its frame's
    # mask into a working buffer first
    _, _, msem = resident_frames(frames, ids=False)
    wm = DeviceBuffer(NPX)

    def sem(k):
        i = k % len(frames)
        wm.copy_from(msem.ptr + i * NPX, NPX, stream=vol.stream)
        vol.parse_frame_dev(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, wm.ptr, Es[i])

    elapsed_s, _, tc_s = timed_integrate(vol, sem, Kf, 2)
    st_s = vol.state()
    res = {
        "workload": "C4 on one GPU: " + C4_SPEC + " (144 GiB)",
        "value": round(1024 ** 3 * K / elapsed / 1e6, 2), "unit": "Mvoxel-updates/s",
        "ms_per_step": round(elapsed * 1e3 / K, 4), "steps": K,
        "integrate_kernel_ms": round(tm.integrate_ms / max(tm.n_integrate, 1), 4),
        "prep_ms": round(tm.prep_ms / max(tm.n_prep, 1), 4),
        "final_render_ms": round(render_ms, 4),
        "per_frame_view": {"value": round(1024 ** 3 * Kf / elapsed_f / 1e6, 2), "unit": "Mvoxel-updates/s",
                           "ms_per_step": round(elapsed_f * 1e3 / Kf, 4), "steps": Kf,
                           "step": "integrate + one label raycast view per frame"},
        "per_frame_semantic": {"value": round(1024 ** 3 * Kf / elapsed_s / 1e6, 2), "unit": "Mvoxel-updates/s",
                               "frames_per_s": round(Kf / elapsed_s, 1),
                               "ms_per_step": round(elapsed_s * 1e3 / Kf, 4), "steps": Kf,
                               "step": "association raycast + relabel + integrate per frame",
                               # the decision's exact f32 path over the last pass of Kf frames
                               "assoc_decisions": int(tc_s.n_assoc),
                               "exact_frames": int(tc_s.assoc_exact_frames),
                               "exact_rows": int(tc_s.assoc_exact_rows),
                               "pos_max": round(float(tc_s.assoc_pos_max), 6),
                               "n_obs_at_end": int(st_s.n_obs), "num_objs_at_end": int(st_s.num_objs),
                               "state_note": "every integrated frame (the integrate-only steps before this leg "
                                             "included) advances n_obs, as tsdf.cu:218-220 (ABI 12)"},
        "touched_per_frame": int(tc.touched / K),
        "device_gib": round(vol.state().device_bytes / 2 ** 30, 1),
    }
    out.free()
    for b in (dbuf, rbuf, mbuf, msem, wm):
        b.free()
    vol.close()
    return res


def run_c4_dist(semtsdf, L, rank, world, local, pg, frames, f0, K, warmup, chunk, async_prepass=True):
    """C4 strong scaling: rank r integrates shard r of the 1024^3 volume (no collective on
    that path); after the K frames one label raycast view is composited across the shards
    (DistShardGroup: RCCL all-reduce MIN between the protocol steps).  Then the per-frame
    variant: the composite after every frame."""
    import torch

    from semtsdf.shard import DistShardGroup

    p = c4_params(semtsdf, L, f0, world, rank, chunk)
    vol = semtsdf.Volume(p, local)
    grp = DistShardGroup(vol, exchange=os.environ.get("BENCH_C4_EXCHANGE", "min"))
    dbuf, rbuf, mbuf = resident_frames(frames, ids=True)
    Es = [(fr.w2c @ f0.c2w).astype(np.float32) for fr in frames]
    mean_m = float(np.mean(f0.depth[f0.depth > 0]) / 5000.0)
    out = torch.empty(NPX * 3, dtype=torch.uint8, device=torch.device("cuda", local))
    torch.cuda.synchronize()

    def integ(k):
        i = k % len(frames)
        if async_prepass:  # as the C3 step: the prepass beside the previous frame's integrate
            vol.integrate_dev_async(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, mbuf.ptr + i * NPX, Es[i])
        else:
            vol.integrate_dev(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, mbuf.ptr + i * NPX, Es[i])

    def view(k=0):
        s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * k, mean_m)
        grp.raycast_dev(s2w, c, L.RENDER_LABEL, out.data_ptr())

    elapsed, tm, tc = timed_integrate(vol, integ, K, warmup, pg, local, finish=view)
    t_max = max_over_ranks(pg, local, elapsed)
    kern = tm.integrate_ms / max(tm.n_integrate, 1)
    prep = tm.prep_ms / max(tm.n_prep, 1)
    # the composite alone, timed around one view (barriers on both sides)
    vol.sync()
    barrier(pg, local)
    tc0 = time.perf_counter()
    view()
    vol.sync()
    barrier(pg, local)
    comp = max_over_ranks(pg, local, time.perf_counter() - tc0)
    Kf = max(4, K // 3)
    elapsed_f, _, _ = timed_integrate(vol, lambda k: (integ(k), view(k)), Kf, 1, pg, local)
    # the semantic frame across the shards: the association ray protocol (RCCL all-reduce MIN
    # between its steps) + all-reduce SUM of the partial tables + relabel, then the integrate
    msem = torch.from_numpy(np.stack([fr.mask.reshape(-1) for fr in frames])).to(out.device)
    wm = torch.empty(NPX, dtype=torch.uint8, device=out.device)

    def sem(k):
        i = k % len(frames)
        wm.copy_(msem[i])
        grp.parse_frame_dev(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, wm.data_ptr(), Es[i])

    elapsed_s, _, _ = timed_integrate(vol, sem, Kf, 2, pg, local)
    touched, gated = tc.touched / K, tc.gated / K
    rank_bytes = 16.0 * touched + 14.0 * gated + 6.0 * NPX  # SURVEY §8d rule, this rank's voxels
    kerns = gather_over_ranks(pg, local, kern)
    bytes_all = gather_over_ranks(pg, local, rank_bytes)
    res = {
        "elapsed": t_max,
        "integrate_kernel_ms_max": max(kerns),
        "integrate_kernel_ms_ranks": kerns,
        "algorithmic_bytes_ranks": bytes_all,
        "prep_ms_max": max_over_ranks(pg, local, prep),
        "composite_ms": comp * 1e3,
        "per_frame_elapsed": max_over_ranks(pg, local, elapsed_f), "per_frame_steps": Kf,
        "semantic_elapsed": max_over_ranks(pg, local, elapsed_s),
        "touched_per_frame": sum_over_ranks(pg, local, touched),
        "gated_per_frame": sum_over_ranks(pg, local, gated),
        "local_planes": int(vol.state().local_dim[2]),
        "device_gib": round(vol.state().device_bytes / 2 ** 30, 1),
    }
    for b in (dbuf, rbuf, mbuf):
        b.free()
    vol.close()
    return res


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--frames", type=int, default=16, help="distinct synthetic frames cycled through")
    ap.add_argument("--c4-chunk", type=int, default=47,
                    help="Z-slab chunk of the C4 shards (planes; chunk + halo = three 16-plane units)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="skip pipeline, orbit, C2 and C4-single")
    ap.add_argument("--no-c4", action="store_true", help="skip the 1024^3 single-GPU C4 measurement")
    ap.add_argument("--no-cull", action="store_true", help="debug: disable unit culling")
    ap.add_argument("--async-prepass", action="store_true", default=True,
                    help="C3 step: frame k's prepass (depth pyramid + unit cull) on the volume's prep stream beside "
                         "frame k-1's integrate (semtsdf_integrate_dev_async; the default: 0.094 against 0.097 ms per "
                         "step, profiles/r04/ab_async_prepass_c3.txt)")
    ap.add_argument("--sync-prepass", dest="async_prepass", action="store_false",
                    help="C3 step: the prepass on the volume's stream in front of its integrate")
    ap.add_argument("--only", choices=["pipeline", "masks", "c2", "c4"], default=None,
                    help="debug: run one section alone and print its record")
    ap.add_argument("--cpu-planes", type=int, default=64)
    ap.add_argument("--cpu-slabs", type=int, default=10)
    ap.add_argument("--cpu-workers", type=int, default=0, help="N-core CPU baseline workers (0 = host cores)")
    ap.add_argument("--c2-traffic-json", default=os.path.join(ROOT, "profiles", "traffic_c2_latest.json"),
                    help="PMC bytes per launch of the C2 integrate (tools/diag_c2.sh)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes of the integrate kernel from rocprofv3 PMC (tools/traffic.py)")
    args = ap.parse_args()

    rank, world, local, pg = dist_setup(args.gpus)
    # probe: one rank's shard of an N-way C4 volume in a single process (per-rank integrate
    # cost, measurable on one GPU); not a scaling result
    emu_world = int(os.environ.get("BENCH_EMULATE_WORLD", "0"))
    emu_rank = int(os.environ.get("BENCH_EMULATE_RANK", "0"))
    import semtsdf
    from semtsdf import _lib as L
    from semtsdf.synth import SyntheticStream

    semtsdf.load()
    t_gen = time.perf_counter()
    stream = SyntheticStream(seed=1, noise=True)
    f0 = stream.frame(0)
    frames = [stream.frame(k) for k in range(1, args.frames + 1)]
    log(f"[bench rank {rank}] generated {len(frames) + 1} frames in {time.perf_counter() - t_gen:.1f}s")

    if world > 1:
        # the same workload on one GPU, timed in this run before any shard is allocated (rank
        # 0, whole 1024^3 volume; the other ranks wait): the base of speedup_vs_1gpu
        base = None
        if rank == 0 and not args.no_c4:
            base = run_c4_single(semtsdf, L, local, frames, f0, args.steps, args.warmup, args.async_prepass)
            log(f"[bench rank 0] C4 on one GPU: {base['ms_per_step']:.4f} ms per step")
        barrier(pg, local)
        r = run_c4_dist(semtsdf, L, rank, world, local, pg, frames, f0, args.steps, args.warmup, args.c4_chunk,
                        args.async_prepass)
        if rank == 0:
            value = 1024 ** 3 * args.steps / r["elapsed"] / 1e6
            kf = r["per_frame_steps"]
            slow = int(np.argmax(r["integrate_kernel_ms_ranks"]))
            kms = r["integrate_kernel_ms_ranks"][slow]
            sb = r["algorithmic_bytes_ranks"][slow]
            ach = sb / (kms * 1e-3) / 1e9
            pf_value = 1024 ** 3 * kf / r["per_frame_elapsed"] / 1e6
            rec = {
                "metric": METRIC, "value": round(value, 2), "unit": "Mvoxel-updates/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["elapsed"] * 1e3 / args.steps, 4),
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic",
                "config": {"workload": "C4 (not C3: the N=1 line's value is the 512^3 C3 workload, so value_N / "
                                       "value_1 is no speed-up; use speedup_vs_1gpu) -- " + C4_SPEC +
                                       "; Z-slab sharded over the ranks (interleaved chunks), composite by RCCL "
                                       "all-reduce MIN between protocol steps",
                           "volume": [1024, 1024, 1024], "z_chunk": args.c4_chunk, "frames_cycled": len(frames),
                           "parallelism": f"zslab{world}"},
                "speedup_vs_1gpu": round(value / base["value"], 3) if base else None,
                "c4_1gpu_in_run": base,
                "frames_per_s": round(args.steps / r["elapsed"], 1),
                "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                             "rank": slow, "algorithmic_bytes_per_launch": int(sb),
                             "bytes_rule": "16 N_touch + 14 N_gate + 6 W H of the slowest rank's voxels (SURVEY "
                                           "§8d) / that rank's integrate kernel time, against one GPU's peak"},
                "integrate_kernel_ms_ranks": [round(x, 4) for x in r["integrate_kernel_ms_ranks"]],
                "integrate_kernel_ms_max_rank": round(r["integrate_kernel_ms_max"], 4),
                "prep_ms_max_rank": round(r["prep_ms_max"], 4),
                "final_composite_ms": round(r["composite_ms"], 4),
                "per_frame_composite": {"value": round(pf_value, 2), "unit": "Mvoxel-updates/s",
                                        "frames_per_s": round(kf / r["per_frame_elapsed"], 1),
                                        "ms_per_step": round(r["per_frame_elapsed"] * 1e3 / kf, 4), "steps": kf,
                                        "step": "integrate + one composited label view per frame",
                                        "speedup_vs_1gpu": round(pf_value / base["per_frame_view"]["value"], 3)
                                        if base else None},
                "per_frame_semantic": {"value": round(1024 ** 3 * kf / r["semantic_elapsed"] / 1e6, 2),
                                       "unit": "Mvoxel-updates/s", "frames_per_s": round(kf / r["semantic_elapsed"], 1),
                                       "ms_per_step": round(r["semantic_elapsed"] * 1e3 / kf, 4), "steps": kf,
                                       "step": "sharded association protocol + relabel + integrate per frame",
                                       "speedup_vs_1gpu": round((1024 ** 3 * kf / r["semantic_elapsed"] / 1e6) /
                                                                base["per_frame_semantic"]["value"], 3)
                                       if base else None},
                "touched_per_frame": int(r["touched_per_frame"]),
                "gated_per_frame": int(r["gated_per_frame"]),
                "local_planes_rank0": r["local_planes"], "device_gib_rank0": r["device_gib"],
            }
            print(json.dumps(rec), flush=True)
        pg.destroy_process_group()
        return

    D = args.dim
    p = place(semtsdf, L, D, f0)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR | (L.F_NO_CULL if args.no_cull else 0)
    if args.only:
        if args.only == "pipeline":
            r = dict(zip(("pipeline", "orbit"), run_pipeline(semtsdf, L, p, local)))
        elif args.only == "masks":
            r = run_mask_overlap(semtsdf, L, p, local, frames, f0)
        elif args.only == "c2":
            r = run_c2(semtsdf, L, local, frames, f0, args.steps, args.warmup, args.c2_traffic_json,
                       args.async_prepass)
        else:
            r = run_c4_single(semtsdf, L, local, frames, f0, args.steps, args.warmup, args.async_prepass)
        print(json.dumps({"only": args.only, args.only: r}), flush=True)
        return
    if emu_world > 1:
        p = c4_params(semtsdf, L, f0, emu_world, emu_rank, args.c4_chunk)
    # CPU baseline first: the forked N-core workers then start from a process that has not
    # touched the GPU yet.
    cpu = cpu_n = None
    if emu_world <= 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(frames, p, f0, args.cpu_planes, args.cpu_slabs, 1)
        nw = args.cpu_workers or host_cores()
        if nw > 1:
            cpu_n = cpu_baseline(frames, p, f0, args.cpu_planes, max(args.cpu_slabs, nw), nw)
        log(f"[bench] cpu baseline 1 core {cpu['value']:.1f} Mvox/s"
            + (f", {nw} cores {cpu_n['value']:.1f} Mvox/s" if cpu_n else ""))

    vol = semtsdf.Volume(p, local)
    st0 = vol.state()
    log(f"[bench] volume {list(p.dim)} local {list(st0.local_dim)} device bytes {st0.device_bytes / 2**30:.2f} GiB")
    dbuf, rbuf, mbuf = resident_frames(frames, ids=True)  # globally consistent ids: integrate-only step
    Es = [(fr.w2c @ f0.c2w).astype(np.float32) for fr in frames]
    vol.sync()

    def step(k):
        i = k % len(frames)
        if args.async_prepass:  # the prepass on the volume's prep stream (semtsdf_integrate_dev_async)
            vol.integrate_dev_async(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, mbuf.ptr + i * NPX, Es[i])
        else:
            vol.integrate_dev(dbuf.ptr + i * NPX * 2, rbuf.ptr + i * NPX * 3, mbuf.ptr + i * NPX, Es[i])

    elapsed, tm, tc = timed_integrate(vol, step, args.steps, args.warmup)
    kern_ms = tm.integrate_ms / max(tm.n_integrate, 1)
    prep_ms = tm.prep_ms / max(tm.n_prep, 1)
    touched = tc.touched / args.steps
    gated = tc.gated / args.steps
    bytes_per_launch = 16.0 * touched + 14.0 * gated + 6.0 * NPX
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    voxels = int(p.dim[0]) * int(p.dim[1]) * int(p.dim[2]) if emu_world <= 1 else (1024 ** 3) // emu_world
    value = voxels * args.steps / elapsed / 1e6
    traffic, traffic_src = read_traffic(args.traffic_json, D, 1)
    live_units = tc.bricks / args.steps
    free_units = tc.free_units / args.steps
    full_units = tc.full_units / args.steps
    lazy = tc.lazy_voxels / args.steps
    vol.close()
    for b in (dbuf, rbuf, mbuf):
        b.free()

    pipeline = orbit = c2 = c4 = masks = None
    if not args.no_pipeline and emu_world <= 1:
        pipeline, orbit = run_pipeline(semtsdf, L, p, local)
        try:  # an auxiliary leg: a failure is reported in the line, not fatal to it
            masks = run_mask_overlap(semtsdf, L, p, local, frames, f0)
        except Exception as e:  # pragma: no cover
            masks = {"error": repr(e)}
        c2 = run_c2(semtsdf, L, local, frames, f0, args.steps, args.warmup, args.c2_traffic_json,
                       args.async_prepass)
        if not args.no_c4:
            c4 = run_c4_single(semtsdf, L, local, frames, f0, args.steps, args.warmup, args.async_prepass)
    copy_bw = copy_bandwidth(local) if not args.no_pipeline else None

    rec = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mvoxel-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": "C3: 512^3 semantic TSDF integrate (sdf f32, weight i32, colour u8x3, 32-bin u32 instance "
                        "histogram), synthetic 640x480 depth+RGB+mask stream (seed 1, noise on), frames resident in "
                        "HBM" if emu_world <= 1 else
                        f"probe: shard {emu_rank} of the {emu_world}-way C4 volume (integrate only)",
            "volume": list(p.dim),
            "frames_cycled": len(frames),
        },
        "frames_per_s": pipeline["frames_per_s"] if pipeline else None,
        "integrate_frames_per_s": round(args.steps / elapsed, 2),
        "prepass": ("frame k's depth pyramid + unit cull on the volume's prep stream beside frame k-1's integrate "
                    "(semtsdf_integrate_dev_async)") if args.async_prepass else "in front of the frame's integrate",
        "integrate_kernel_ms": round(kern_ms, 4),
        "prep_ms": round(prep_ms, 4),
        "prep_exposed_ms": round(elapsed * 1e3 / args.steps - kern_ms, 4),
        "prep_note": ("prep_ms: the prepass kernels' own span, overlapping the previous integrate on the prep stream; "
                      "prep_exposed_ms: step time not covered by the integrate kernel") if args.async_prepass else
                     "prep_ms: the prepass kernels in front of the integrate",
        "touched_per_frame": int(touched),
        "gated_per_frame": int(gated),
        "live_units_per_frame": int(live_units),
        "free_units_per_frame": int(free_units),
        "full_free_units_per_frame": int(full_units),
        "lazy_weight_voxels_per_frame": int(lazy),
        "touched_mvox_per_s": round(touched / (kern_ms * 1e-3) / 1e6, 1),
        "touched_lines_per_frame": int(tc.touched_lines / args.steps),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "bytes_rule": "16 N_touch + 14 N_gate + 6 W H (SURVEY §8d, the reference's storage types)",
        },
        "cpu_baseline": cpu,
        "cpu_baseline_ncores": cpu_n,
        "hbm_copy_gbs": round(copy_bw, 1) if copy_bw else None,
        "pipeline": pipeline,
        "orbit": orbit,
        "mask_producer": masks,
        "c2": c2,
        "c4_single_gpu": c4,
    }
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
