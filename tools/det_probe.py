"""Probe (not part of the product): Mask R-CNN producer time per frame under MIOpen settings.
Usage: python tools/det_probe.py {cl|nchw} {bench0|bench1} [fp32]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from semtsdf import maskrcnn as MR  # noqa: E402
from semtsdf.synth import SyntheticStream  # noqa: E402

layout, bench = sys.argv[1], sys.argv[2]
dt = sys.argv[3] if len(sys.argv) > 3 else "bf16"
fp32 = dt == "fp32"
torch.backends.cudnn.benchmark = bench == "bench1"
dev = torch.device("cuda", 0)
img = torch.from_numpy(SyntheticStream(seed=1, noise=True).frame(0).rgb).to(dev)
cfg = MR.Config(DTYPE={"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[dt])
m = MR.MaskRCNN(cfg, seed=0).to(dev).to(cfg.DTYPE).eval()
MR.CHANNELS_LAST = layout == "cl"
t0 = time.perf_counter()
m.detect(img, compact=False)
torch.cuda.synchronize()
t1 = time.perf_counter()
for _ in range(3):
    m.detect(img, compact=False)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    m.detect(img, compact=False)
e1.record()
e1.synchronize()
print(f"{layout} {bench} {dt}: first call {t1 - t0:.1f} s, {e0.elapsed_time(e1) / 10:.2f} ms per detect", flush=True)
