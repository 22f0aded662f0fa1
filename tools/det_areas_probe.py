"""Probe: the C5 producer's per-frame detections, box and mask areas, and how many pass the
dmask.py area filter (semtsdf_masks_to_labels, min_area 2000) -- instrumentation for the bench's C5 leg."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))
from semtsdf import maskrcnn as MR  # noqa: E402
from semtsdf.masks import masks_to_labels_dev  # noqa: E402
from semtsdf.synth import SyntheticStream  # noqa: E402

dev = torch.device("cuda", 0)
st = SyntheticStream(seed=1, noise=True)
imgs = [torch.from_numpy(st.frame(k).rgb).to(dev) for k in range(4)]
cfg = MR.Config(DTYPE=torch.float16)
m = MR.MaskRCNN(cfg, seed=0).to(dev).to(cfg.DTYPE).eval()
m.calibrate(dev, imgs[0])
for k, im in enumerate(imgs):
    out = m.detect(im)
    r = out["rois"].cpu().numpy()
    ms = out["masks"].cpu().numpy()
    box_a = (r[:, 2] - r[:, 0]) * (r[:, 3] - r[:, 1])
    mask_a = ms.reshape(-1, ms.shape[2]).sum(0)
    labels = torch.zeros(480 * 640, dtype=torch.uint8, device=dev)
    kept = masks_to_labels_dev(out["masks"].data_ptr(), 640, 480, ms.shape[2], labels.data_ptr(),
                               stream=torch.cuda.current_stream(dev).cuda_stream, want_count=True)
    print(f"frame {k}: {len(r)} detections, box areas {np.sort(box_a)[::-1][:12].tolist()}, "
          f"mask areas {np.sort(mask_a)[::-1][:12].tolist()}, kept {kept}, label pixels {int((labels > 0).sum())}",
          flush=True)
