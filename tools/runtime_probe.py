"""Which HIP runtime does libsemtsdf bind to when torch is imported first, and does the
engine run on it?  (torch wheels bundle their own libamdhip64 with the same SONAME.)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))
mode = sys.argv[1] if len(sys.argv) > 1 else "torch-first"
if mode == "torch-first":
    import torch

    torch.cuda.init()
    x = torch.ones(4, device="cuda")
import __graft_entry__ as g  # noqa: E402

g.smoke()
maps = open("/proc/self/maps").read().splitlines()
libs = sorted({ln.split()[-1] for ln in maps if "libamdhip64" in ln or "libhsa-runtime64" in ln})
print("mode", mode, "runtimes:", libs)
if mode == "torch-first":
    print("torch still ok:", float((x * 2).sum().item()))
