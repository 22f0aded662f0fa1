"""Host time of one frame's H2D upload (depth, RGB, mask from pinned memory) by method, with
the GPU idle and with the GPU busy (a long kernel queued first): torch copy_(non_blocking)
on a side stream, semtsdf_memcpy (hipMemcpyAsync) on a side stream, and one combined copy.
Usage: python3 tools/upload_probe.py"""
import ctypes as C
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "slam-maskrcnn_amd"))
import semtsdf  # noqa: E402
from semtsdf import _lib as L  # noqa: E402

NPX = 640 * 480
lib = L.load()
dev = torch.device("cuda", 0)
h = torch.empty(NPX * 6, dtype=torch.uint8).pin_memory()
d = torch.empty(NPX * 6, dtype=torch.uint8, device=dev)
big_a = torch.empty(1 << 28, dtype=torch.float32, device=dev)
big_b = torch.empty_like(big_a)
cs = torch.cuda.Stream(device=dev)
print("pinned:", h.is_pinned())


def busy():
    for _ in range(4):
        big_b.copy_(big_a)  # ~1 GB each on the default stream


def torch3():
    with torch.cuda.stream(cs):
        d[:NPX * 2].copy_(h[:NPX * 2], non_blocking=True)
        d[NPX * 2:NPX * 5].copy_(h[NPX * 2:NPX * 5], non_blocking=True)
        d[NPX * 5:].copy_(h[NPX * 5:], non_blocking=True)


def lib3():
    s = C.c_void_p(cs.cuda_stream)
    for a, b in ((0, NPX * 2), (NPX * 2, NPX * 5), (NPX * 5, NPX * 6)):
        L.check(lib.semtsdf_memcpy(C.c_void_p(d.data_ptr() + a), C.c_void_p(h.data_ptr() + a), b - a, 1, s))


def lib1():
    L.check(lib.semtsdf_memcpy(C.c_void_p(d.data_ptr()), C.c_void_p(h.data_ptr()), NPX * 6, 1,
                               C.c_void_p(cs.cuda_stream)))


ev = torch.cuda.Event()


def lib1_wait():  # after an event recorded behind the busy work (the pipeline's ring slot reuse)
    ev.record(torch.cuda.current_stream())
    cs.wait_event(ev)
    lib1()


def lib1_wait_done():  # after an event that already completed
    cs.wait_event(ev)
    lib1()


hb = [torch.empty(NPX * 6, dtype=torch.uint8).pin_memory() for _ in range(8)]
kk = [0]


def lib1_rot():  # a different pinned source buffer each call
    kk[0] = (kk[0] + 1) % 8
    L.check(lib.semtsdf_memcpy(C.c_void_p(d.data_ptr()), C.c_void_p(hb[kk[0]].data_ptr()), NPX * 6, 1,
                               C.c_void_p(cs.cuda_stream)))


hbig = torch.empty((64, NPX * 6), dtype=torch.uint8).pin_memory()


def lib1_big():  # frame k of one large pinned allocation (bench.run_pipeline's layout)
    kk[0] = (kk[0] + 1) % 64
    L.check(lib.semtsdf_memcpy(C.c_void_p(d.data_ptr()), C.c_void_p(hbig[kk[0]].data_ptr()), NPX * 6, 1,
                               C.c_void_p(cs.cuda_stream)))


hs = torch.cuda.Stream(device=dev, priority=-1)


def lib1_wait_hi():  # after an event recorded behind work on a high-priority stream
    with torch.cuda.stream(hs):
        big_b.copy_(big_a)
    ev.record(hs)
    cs.wait_event(ev)
    lib1()


vlib = None


def lib1_wait_libstream():  # after an event recorded on the library's own volume stream
    global vlib
    if vlib is None:
        p = semtsdf.default_params(64, (520.9, 521.0, 325.1, 249.7), 640, 480)
        vlib = semtsdf.Volume(p, 0)
    vs = torch.cuda.ExternalStream(vlib.stream, device=dev)
    with torch.cuda.stream(vs):
        big_b.copy_(big_a)
    ev.record(vs)
    cs.wait_event(ev)
    lib1()


for name, fn in (("memcpy after hi-prio", lib1_wait_hi), ("memcpy after lib stream", lib1_wait_libstream),
                 ("memcpy from big pinned", lib1_big), ("torch copy_ x3", torch3), ("semtsdf_memcpy x3", lib3), ("semtsdf_memcpy x1", lib1),
                 ("memcpy after wait", lib1_wait), ("memcpy after done ev", lib1_wait_done),
                 ("memcpy rotating src", lib1_rot)):
    for state in ("idle", "busy"):
        ts = []
        for _ in range(20):
            torch.cuda.synchronize()
            if state == "busy":
                busy()
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        torch.cuda.synchronize()
        ts.sort()
        print(f"{name:18s} GPU {state}: host median {ts[len(ts) // 2] * 1e6:8.1f} us, max {ts[-1] * 1e6:8.1f} us")
