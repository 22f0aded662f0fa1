"""Benchmark of the semantic TSDF hot path on MI355X (BASELINE.json metric:
"Mvoxel-updates/s + frames/s, 512^3 semantic TSDF @ 640x480").

One step = one frame of the per-frame integrate (src/SfM_CUDA/tsdf.cu:18-70 semantics:
SDF + gated colour + 32-bin instance histogram) over the whole volume, inputs resident
in HBM.  N=1 runs configuration C3 (512^3 semantic, synthetic 640x480 stream with masks).
N>1 ranks (torchrun, one process per GPU) each own an interleaved Z-slab shard of a
512 x 512 x (512 N) volume covering the same physical box (the SfM placement divides
each axis by its own dim, so z resolution grows N-fold) -- every GPU owns 512^3 voxels
and sees the same share of the surface band per frame (weak scaling; Z-slab sharding
needs no collective for integrate).

value = voxels integrated by all ranks / max-over-ranks wall time of the K timed steps.
Extra fields: frames/s of the full per-frame pipeline (association raycast + relabel +
integrate, N=1), render time, the integrate kernel's HBM roofline and the CPU baseline
(NumPy restatement of tsdf.py:78-120 + SfM gate, bounded sample, 1 core).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))

METRIC = "Mvoxel-updates/s + frames/s, 512^3 semantic TSDF @ 640x480"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
KI = (520.9, 521.0, 325.1, 249.7)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup(n_gpus):
    """One process per GPU (torch.distributed.run).  The data path has no collective (each
    rank integrates its own Z-slab shard); the process group only carries the barrier and
    the max/sum of the timings.  Backend: RCCL ("nccl") by default; BENCH_DIST_BACKEND=gloo
    rehearses N ranks on fewer GPUs (device = LOCAL_RANK % device count)."""
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


def copy_bandwidth(device: int, nbytes: int = 1 << 30) -> float:
    """Achievable HBM bandwidth (GB/s, read + write) of a float4 device copy (library kernel),
    for context beside the 8 TB/s spec peak."""
    import ctypes as C

    from semtsdf import _lib as L

    out = C.c_double()
    L.check(L.load().semtsdf_copy_bandwidth(int(device), int(nbytes), 5, C.byref(out)))
    return out.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--frames", type=int, default=16, help="distinct synthetic frames cycled through")
    ap.add_argument("--z-chunk", type=int, default=63)  # 63 + 1 halo plane = 4 half-tile units per chunk
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--no-cull", action="store_true", help="debug: disable brick culling")
    ap.add_argument("--cpu-planes", type=int, default=64)
    ap.add_argument("--cpu-slabs", type=int, default=10)
    ap.add_argument("--cpu-workers", type=int, default=0, help="N-core CPU baseline workers (0 = host cores)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes of the integrate kernel from rocprofv3 PMC (see profiles/)")
    args = ap.parse_args()

    rank, world, local, pg = dist_setup(args.gpus)
    # probe: one rank's shard of an N-way volume in a single process (per-rank cost of the
    # N-GPU weak-scaling run, measurable on one GPU); not a scaling result
    emu_world = int(os.environ.get("BENCH_EMULATE_WORLD", "0"))
    emu_rank = int(os.environ.get("BENCH_EMULATE_RANK", "0"))
    shard_world, shard_rank = (emu_world, emu_rank) if (emu_world > 1 and world == 1) else (world, rank)
    import semtsdf
    from semtsdf import _lib as L
    from semtsdf.synth import SyntheticStream
    from semtsdf.volume import DeviceBuffer

    semtsdf.load()
    D = args.dim
    W, H = 640, 480
    t_gen = time.perf_counter()
    stream = SyntheticStream(seed=1, noise=True)
    f0 = stream.frame(0)
    frames = [stream.frame(k) for k in range(1, args.frames + 1)]
    log(f"[bench rank {rank}] generated {len(frames) + 1} frames in {time.perf_counter() - t_gen:.1f}s")

    p = semtsdf.default_params(D, KI, W, H)
    p.dim[2] = D * shard_world
    semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR | (L.F_NO_CULL if args.no_cull else 0)
    if shard_world > 1:
        p.z_nshards = shard_world
        p.z_shard = shard_rank
        p.z_chunk = args.z_chunk
    # CPU baseline first: the forked N-core workers then start from a process that has not
    # touched the GPU yet.
    cpu = cpu_n = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(frames, p, f0, args.cpu_planes, args.cpu_slabs, 1)
        nw = args.cpu_workers or host_cores()
        if nw > 1:
            cpu_n = cpu_baseline(frames, p, f0, args.cpu_planes, max(args.cpu_slabs, nw), nw)
        log(f"[bench] cpu baseline 1 core {cpu['value']:.1f} Mvox/s"
            + (f", {nw} cores {cpu_n['value']:.1f} Mvox/s" if cpu_n else ""))

    vol = semtsdf.Volume(p, local)
    st0 = vol.state()
    voxels_per_rank = D * D * D  # owned voxels (halo planes are integrated redundantly, not counted)
    log(f"[bench rank {rank}] volume {list(p.dim)} local {list(st0.local_dim)} "
        f"device bytes {st0.device_bytes / 2**30:.2f} GiB")

    # frames resident in HBM
    npx = W * H
    dbuf = DeviceBuffer(len(frames) * npx * 2)
    rbuf = DeviceBuffer(len(frames) * npx * 3)
    mbuf = DeviceBuffer(len(frames) * npx)
    Es = []
    for i, fr in enumerate(frames):
        dbuf.upload(fr.depth, None, i * npx * 2)
        rbuf.upload(fr.rgb, None, i * npx * 3)
        mbuf.upload(fr.gt_ids, None, i * npx)  # globally consistent ids: integrate-only step
        Es.append((fr.w2c @ f0.c2w).astype(np.float32))
    vol.sync()

    def step(k):
        i = k % len(frames)
        vol.integrate_dev(dbuf.ptr + i * npx * 2, rbuf.ptr + i * npx * 3, mbuf.ptr + i * npx, Es[i])

    for k in range(args.warmup):
        step(k)
    vol.sync()
    # timed region: the K steps alone (no timing events on the stream)
    barrier(pg, local)
    vol.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    vol.sync()
    barrier(pg, local)
    t1 = time.perf_counter()
    elapsed = max_over_ranks(pg, local, t1 - t0)

    # kernel-level timing of the same K steps: HIP events on the volume's stream around the
    # prepass (pyramid + cull) and around the integrate kernel
    vol.reset_timing()
    vol.set_instrumentation(events=True, count=False)
    for k in range(args.steps):
        step(args.warmup + k)
    vol.sync()
    tm = vol.timing()
    vol.set_instrumentation(events=False, count=False)
    kern_ms = tm.integrate_ms / max(tm.n_integrate, 1)
    prep_ms = tm.prep_ms / max(tm.n_prep, 1)

    # algorithmic bytes of the same launches (counts are a function of the frame only)
    vol.reset_timing()
    vol.set_instrumentation(events=False, count=True)
    for k in range(args.steps):
        step(args.warmup + k)
    tc = vol.timing()
    vol.set_instrumentation(events=False, count=False)
    touched = tc.touched / args.steps
    gated = tc.gated / args.steps
    bricks = tc.bricks / args.steps
    free_units = tc.free_units / args.steps
    bytes_per_launch = 16.0 * touched + 14.0 * gated + 6.0 * npx
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9

    total_vox = sum_over_ranks(pg, local, float(voxels_per_rank) * args.steps)
    value = total_vox / elapsed / 1e6

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("dim") == D and tj.get("n_gpus", 1) == world:
                traffic = tj.get("bytes_per_launch")
        except Exception:
            traffic = None

    pipeline = None
    if world == 1 and not args.no_pipeline:
        # full per-frame pipeline (SfM launch_kernel order): association raycast + relabel on
        # device, then integrate; per-frame instance labels permuted as Mask R-CNN would emit.
        vol.reset()
        # per-frame detection masks resident in HBM like the depth/RGB frames (a detector
        # on the same GPU hands over device masks); each frame copies its mask into the
        # work buffer the association relabels in place
        dmask = DeviceBuffer(len(frames) * npx)
        for i, fr in enumerate(frames):
            dmask.upload(fr.mask, vol.stream, i * npx)
        mwork = DeviceBuffer(npx)
        n_pipe = max(args.steps, 2 * len(frames))
        vol.parse_frame_dev(dbuf.ptr, rbuf.ptr, mbuf.ptr, Es[0])  # first integrated frame
        for i in range(1, 3):
            mwork.copy_from(dmask.ptr + i * npx, npx, vol.stream)
            vol.parse_frame_dev(dbuf.ptr + i * npx * 2, rbuf.ptr + i * npx * 3, mwork.ptr, Es[i])
        vol.sync()
        vol.reset_timing()
        vol.set_instrumentation(events=True, count=False)
        tp0 = time.perf_counter()
        for k in range(n_pipe):
            i = (3 + k) % len(frames)
            mwork.copy_from(dmask.ptr + i * npx, npx, vol.stream)  # 307 KB per-frame mask
            vol.parse_frame_dev(dbuf.ptr + i * npx * 2, rbuf.ptr + i * npx * 3, mwork.ptr, Es[i])
        vol.sync()
        tp1 = time.perf_counter()
        tp = vol.timing()
        s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.3, float(np.mean(f0.depth[f0.depth > 0]) / 5000.0))
        obuf = DeviceBuffer(npx * 3)
        vol.reset_timing()
        for _ in range(5):
            vol.raycast_dev(s2w, c, L.RENDER_LABEL, obuf.ptr)
        tr = vol.timing()
        st = vol.state()
        pipeline = {
            "frames_per_s": n_pipe / (tp1 - tp0),
            "ms_per_frame": (tp1 - tp0) * 1e3 / n_pipe,
            "assoc_ms_per_frame": tp.assoc_ms / max(tp.n_assoc, 1),
            "integrate_ms_per_frame": tp.integrate_ms / max(tp.n_integrate, 1),
            "render_ms_per_view": tr.render_ms / max(tr.n_render, 1),
            "num_objs": int(st.num_objs),
        }
        obuf.free()
        mwork.free()
        dmask.free()

    copy_bw = None
    if rank == 0 and not args.no_pipeline:
        copy_bw = copy_bandwidth(local)

    if rank == 0:
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
                "workload": "C3: 512^3 semantic TSDF integrate (sdf f32, weight i32, colour u8x3, 32-bin u32 "
                            "instance histogram), synthetic 640x480 depth+RGB+mask stream (seed 1, noise on), "
                            "frames resident in HBM; N>1: interleaved Z-slab shards of 512x512x(512N)",
                "volume": list(p.dim),
                "z_chunk": int(p.z_chunk) if world > 1 else None,
                "frames_cycled": len(frames),
            },
            "frames_per_s": round(args.steps / elapsed, 2),
            "integrate_kernel_ms": round(kern_ms, 4),
            "prep_ms": round(prep_ms, 4),
            "touched_per_frame": int(touched),
            "gated_per_frame": int(gated),
            "live_units_per_frame": int(bricks),
            "free_units_per_frame": int(free_units),
            "touched_mvox_per_s": round(touched / (kern_ms * 1e-3) / 1e6, 1),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
            },
            "cpu_baseline": cpu,
            "cpu_baseline_ncores": cpu_n,
            "hbm_copy_gbs": round(copy_bw, 1) if copy_bw else None,
            "pipeline": pipeline,
        }
        print(json.dumps(rec), flush=True)
    vol.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
