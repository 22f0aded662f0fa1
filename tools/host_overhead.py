"""Host cost of the C3 pipeline loop (bench.run_pipeline's fused frame), per section: the
TUM pose path, the frame's library call, the orbit camera, the upload of a later frame, and
the wall time per frame with the GPU in the loop.
Usage: python3 tools/host_overhead.py [RING] [LAG] [torch|lib]
(upload of frame k + RING - LAG after frame k, into the slot frame k - LAG used)"""
import ctypes as C
import os
import sys
import tempfile
import time

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "slam-maskrcnn_amd"))
import semtsdf  # noqa: E402
from semtsdf import _lib as L  # noqa: E402
from semtsdf import pose as P  # noqa: E402
from semtsdf import tum  # noqa: E402
from semtsdf.synth import SyntheticStream  # noqa: E402

W, H, NPX = 640, 480, 640 * 480
semtsdf.load()
st = SyntheticStream(seed=1, noise=True)
n_all = 64
frames = [st.frame(k) for k in range(n_all)]
with tempfile.TemporaryDirectory() as d:
    gt = os.path.join(d, "groundtruth.txt")
    with open(gt, "w") as f:
        f.write("\n".join(st.tum_lines(n_all)) + "\n")
    traj = tum.read_traj(gt)
p = semtsdf.default_params(512, (520.9, 521.0, 325.1, 249.7), W, H)
semtsdf.place_from_frame(p, frames[0].depth, tum.mean_depth_m(frames[0].depth), L.PLACE_SFM)
p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
dev = torch.device("cuda", 0)
vol = semtsdf.Volume(p, 0)
vstream = torch.cuda.ExternalStream(vol.stream, device=dev)
cstream = torch.cuda.Stream(device=dev)
h_d = torch.empty((n_all, NPX), dtype=torch.int16).pin_memory()
h_r = torch.empty((n_all, NPX * 3), dtype=torch.uint8).pin_memory()
h_m = torch.empty((n_all, NPX), dtype=torch.uint8).pin_memory()
for k, fr in enumerate(frames):
    h_d[k].copy_(torch.from_numpy(fr.depth.reshape(-1).view(np.int16)))
    h_r[k].copy_(torch.from_numpy(fr.rgb.reshape(-1)))
    h_m[k].copy_(torch.from_numpy(fr.mask.reshape(-1)))
ring = int(sys.argv[1]) if len(sys.argv) > 1 else 2
lag = int(sys.argv[2]) if len(sys.argv) > 2 else 0
method = sys.argv[3] if len(sys.argv) > 3 else "torch"
d_d = torch.empty((ring, NPX), dtype=torch.int16, device=dev)
d_r = torch.empty((ring, NPX * 3), dtype=torch.uint8, device=dev)
d_m = torch.empty((ring, NPX), dtype=torch.uint8, device=dev)
h_all = torch.empty((n_all, NPX * 6), dtype=torch.uint8).pin_memory()
d_all = torch.empty((ring, NPX * 6), dtype=torch.uint8, device=dev)
for k, fr in enumerate(frames):
    h_all[k, :NPX * 2].copy_(torch.from_numpy(fr.depth.reshape(-1).view(np.uint8)))
    h_all[k, NPX * 2:NPX * 5].copy_(torch.from_numpy(fr.rgb.reshape(-1)))
    h_all[k, NPX * 5:].copy_(torch.from_numpy(fr.mask.reshape(-1)))
lib = L.load()
print(f"ring {ring} lag {lag} method {method}")
outs = [torch.empty(NPX * 3, dtype=torch.uint8, device=dev) for _ in range(2)]
copied = [torch.cuda.Event() for _ in range(ring)]
used = [torch.cuda.Event() for _ in range(ring)]
mean_m = tum.mean_depth_m(frames[0].depth)
ext0_inv = np.linalg.inv(P.parse_pos(traj[0, 1:]))
acc = {"pose": 0.0, "wait": 0.0, "call": 0.0, "orbit": 0.0, "record": 0.0, "upload": 0.0}


sub = {"u_wait": 0.0, "u_copy": 0.0, "u_rec": 0.0}


def upload(k):
    s = k % ring
    if method in ("lib", "kern"):
        a = time.perf_counter()
        cstream.wait_event(used[s])
        b = time.perf_counter()
        L.check(lib.semtsdf_memcpy(C.c_void_p(d_all[s].data_ptr()), C.c_void_p(h_all[k].data_ptr()), NPX * 6,
                                   4 if method == "kern" else 1, C.c_void_p(cstream.cuda_stream)))
        c = time.perf_counter()
        copied[s].record(cstream)
        e = time.perf_counter()
        sub["u_wait"] += b - a
        sub["u_copy"] += c - b
        sub["u_rec"] += e - c
        return
    with torch.cuda.stream(cstream):
        cstream.wait_event(used[s])
        d_d[s].copy_(h_d[k], non_blocking=True)
        d_r[s].copy_(h_r[k], non_blocking=True)
        d_m[s].copy_(h_m[k], non_blocking=True)
        copied[s].record(cstream)


def ptrs(s):
    if method in ("lib", "kern"):
        b = d_all[s].data_ptr()
        return b, b + NPX * 2, b + NPX * 5
    return d_d[s].data_ptr(), d_r[s].data_ptr(), d_m[s].data_ptr()


def frame(k, timed):
    s = k % ring
    t0 = time.perf_counter()
    E = P.relative_pose(P.parse_pos(traj[k, 1:]), ext0_inv)
    t1 = time.perf_counter()
    vstream.wait_event(copied[s])
    t2 = time.perf_counter()
    s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * (k - 1), mean_m)
    t3 = time.perf_counter()
    pd, pr, pm = ptrs(s)
    vol.parse_frame_view_dev(pd, pr, pm, E, s2w, c, L.RENDER_LABEL, outs[(k - 1) % 2].data_ptr())
    t4 = time.perf_counter()
    used[s].record(vstream)
    t5 = time.perf_counter()
    if k + ring - lag < n_all:
        upload(k + ring - lag)
    t6 = time.perf_counter()
    if timed:
        for key, dt in zip(("pose", "wait", "orbit", "call", "record", "upload"),
                           (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
            acc[key] += dt


for k in range(ring - lag):
    upload(1 + k)
for k in range(1, 8):
    frame(k, False)
vol.sync()
torch.cuda.synchronize()
n = 0
t0 = time.perf_counter()
for k in range(8, n_all):
    frame(k, True)
    n += 1
t_enq = time.perf_counter() - t0
vol.sync()
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"frames {n}: wall {t_all / n * 1e6:.1f} us/frame, host enqueue {t_enq / n * 1e6:.1f} us/frame")
for key, v in acc.items():
    print(f"  {key:7s} {v / n * 1e6:7.1f} us/frame")
for key, v in sub.items():
    print(f"  {key:7s} {v / (n + 7 + ring) * 1e6:7.1f} us/call (all uploads)")
# the library call alone, GPU idle between calls (no queueing behind the GPU)
tt = []
for k in range(8, 24):
    vol.sync()
    torch.cuda.synchronize()
    s = k % ring
    E = P.relative_pose(P.parse_pos(traj[k, 1:]), ext0_inv)
    s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * (k - 1), mean_m)
    a = time.perf_counter()
    pd, pr, pm = ptrs(s)
    vol.parse_frame_view_dev(pd, pr, pm, E, s2w, c, L.RENDER_LABEL, outs[(k - 1) % 2].data_ptr())
    tt.append(time.perf_counter() - a)
print(f"library call on an idle GPU: median {np.median(tt) * 1e6:.1f} us")
vol.close()
