"""Mask R-CNN producer in PyTorch-ROCm.

The reference's detector is matterport's Keras/TensorFlow Mask R-CNN (Mask_RCNN/mrcnn/model.py) run
with COCO weights by Mask_RCNN/dmask.py and mask_process.py.  This module restates its inference graph
(`MaskRCNN.build`, mode "inference", model.py:1833-2053) layer for layer in PyTorch, fp16 or bf16
convolutions on MIOpen for the backbone and heads (`Config.DTYPE`; the bench's producer runs fp16), f32
box arithmetic, and the greedy NMS and the PyramidROIAlign as HIP kernels (libsemtsdf_det.so,
include/semtsdf_det.h); `detect` returns what model.py:2436-2492 returns
(rois, class_ids, scores, masks[H, W, N]), on the device, and feeds semtsdf_masks_to_labels (the
dmask.py rule) without leaving HBM.

Weights: the COCO checkpoint (mask_rcnn_coco.h5) is not available offline, so the network is
random-initialised (seeded) with the reference's architecture and shapes; the detections are
therefore arbitrary but the work per frame (backbone, RPN, 1000 proposals, heads, NMS, unmold) is the
reference detector's.

Reference anchors (file:line): config mrcnn/config.py:50-204 (+ COCO NUM_CLASSES 81); resnet_graph
model.py:177-216; FPN model.py:1900-1925; rpn_graph model.py:835-876; generate_pyramid_anchors
utils.py:588-648; ProposalLayer model.py:261-342; PyramidROIAlign model.py:350-459; fpn_classifier_graph
model.py:905-956; refine_detections_graph model.py:689-784; build_fpn_mask_graph model.py:959-1012;
mold_inputs / unmold_detections / detect model.py:2332-2492; resize_image utils.py:392-497; unmold_mask
utils.py:565-586; norm_boxes / denorm_boxes utils.py:858-889.

Restated, not bit-identical (no TensorFlow or scikit-image here): image resizing and mask unmolding
use torch bilinear interpolation (skimage.transform.resize order=1 in the reference); crop_and_resize
is bilinear sampling with the same sample positions and a zero value for samples outside the map.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, field

import numpy as np

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")  # no per-shape tuning sweep on the first frame

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

_ROOT = os.path.dirname(os.path.abspath(__file__))
DET_LIB = os.path.join(_ROOT, "libsemtsdf_det.so")
# NCHW activations: MIOpen's immediate mode runs them at 10.8 ms per 1024x1024 frame against 28.7 ms for
# NHWC (8.9 ms only after a 30-s per-shape find with torch.backends.cudnn.benchmark; tools/det_probe.py)
CHANNELS_LAST = False
ROI_ALIGN_HIP = True  # the device ROI align (libsemtsdf_det.so); False: the PyTorch grid_sample formulation


@dataclass
class Config:
    """mrcnn/config.py:50-204 with samples/coco CocoConfig (81 classes), inference, one image."""
    BACKBONE: str = "resnet101"
    BACKBONE_STRIDES: tuple = (4, 8, 16, 32, 64)
    NUM_CLASSES: int = 81
    RPN_ANCHOR_SCALES: tuple = (32, 64, 128, 256, 512)
    RPN_ANCHOR_RATIOS: tuple = (0.5, 1, 2)
    RPN_ANCHOR_STRIDE: int = 1
    RPN_NMS_THRESHOLD: float = 0.7
    PRE_NMS_LIMIT: int = 6000  # model.py:287
    POST_NMS_ROIS_INFERENCE: int = 1000
    IMAGE_MIN_DIM: int = 800
    IMAGE_MAX_DIM: int = 1024
    MEAN_PIXEL: tuple = (123.7, 116.8, 103.9)
    POOL_SIZE: int = 7
    MASK_POOL_SIZE: int = 14
    TOP_DOWN_PYRAMID_SIZE: int = 256
    FC_LAYERS_SIZE: int = 1024
    RPN_BBOX_STD_DEV: tuple = (0.1, 0.1, 0.2, 0.2)
    BBOX_STD_DEV: tuple = (0.1, 0.1, 0.2, 0.2)
    DETECTION_MAX_INSTANCES: int = 100
    DETECTION_MIN_CONFIDENCE: float = 0.7
    DETECTION_NMS_THRESHOLD: float = 0.3
    DTYPE: torch.dtype = field(default=torch.bfloat16)


# ---------------------------------------------------------------------------------------- NMS
_det = None


def _det_lib():
    global _det
    if _det is None:
        if not os.path.exists(DET_LIB):
            raise RuntimeError(f"{DET_LIB} missing: run __graft_entry__.build() (no CPU fallback)")
        lib = C.CDLL(DET_LIB)
        lib.semtsdf_det_nms_workspace.restype = C.c_size_t
        lib.semtsdf_det_nms_workspace.argtypes = [C.c_int]
        lib.semtsdf_det_nms.restype = C.c_int
        lib.semtsdf_det_nms.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p]
        lib.semtsdf_det_roi_align.restype = C.c_int
        lib.semtsdf_det_roi_align.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int,
                                              C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                              C.c_void_p]
        _det = lib
    return _det


def nms_sorted(boxes: torch.Tensor, iou_threshold: float, max_out: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Greedy NMS of device boxes [n, 4] (y1, x1, y2, x2) sorted by descending score (the HIP kernels
    of libsemtsdf_det.so): returns (keep [max_out] int32 with -1 past the count, count [1] int32), both
    on the device, asynchronous on the current stream."""
    if boxes.device.type != "cuda":
        raise RuntimeError("nms_sorted runs on the GPU (libsemtsdf_det.so); no CPU fallback")
    lib = _det_lib()
    b = boxes.to(torch.float32).contiguous()
    n = int(b.shape[0])
    keep = torch.empty(max(max_out, 1), dtype=torch.int32, device=b.device)
    count = torch.empty(1, dtype=torch.int32, device=b.device)
    work = torch.empty(int(lib.semtsdf_det_nms_workspace(n)), dtype=torch.uint8, device=b.device)
    rc = lib.semtsdf_det_nms(C.c_void_p(b.data_ptr()), n, float(iou_threshold), int(max_out),
                             C.c_void_p(keep.data_ptr()), C.c_void_p(count.data_ptr()), C.c_void_p(work.data_ptr()),
                             C.c_void_p(torch.cuda.current_stream(b.device).cuda_stream))
    if rc:
        raise RuntimeError(f"semtsdf_det_nms failed ({rc})")
    return keep[:max_out], count


def roi_align_dev(rois: torch.Tensor, lvl: torch.Tensor, feats, pool: int) -> torch.Tensor:
    """PyramidROIAlign on the device (the HIP kernel of libsemtsdf_det.so): rois [n, 4] normalised, lvl
    [n] in 2..5, feats the four levels [1, C, H, W] in fp16 or bf16 -> [n, C, pool, pool] in their dtype,
    asynchronous on the current stream.  Each roi reads only its own level."""
    lib = _det_lib()
    fs = [f.contiguous() for f in feats]
    dt = {torch.float16: 0, torch.bfloat16: 1}[fs[0].dtype]
    n, Cn = int(rois.shape[0]), int(fs[0].shape[1])
    out = torch.empty((n, Cn, pool, pool), dtype=fs[0].dtype, device=rois.device)
    r = rois.to(torch.float32).contiguous()
    lv = lvl.to(torch.int32).contiguous()
    ptrs = (C.c_void_p * 4)(*[f.data_ptr() for f in fs])
    H = (C.c_int * 4)(*[int(f.shape[2]) for f in fs])
    W = (C.c_int * 4)(*[int(f.shape[3]) for f in fs])
    rc = lib.semtsdf_det_roi_align(ptrs, H, W, Cn, C.c_void_p(r.data_ptr()), C.c_void_p(lv.data_ptr()), n, int(pool),
                                   dt, C.c_void_p(out.data_ptr()), C.c_void_p(torch.cuda.current_stream(rois.device).cuda_stream))
    if rc:
        raise RuntimeError(f"semtsdf_det_roi_align failed ({rc})")
    return out


# ---------------------------------------------------------------------------------- anchors
def generate_pyramid_anchors(scales, ratios, feature_shapes, feature_strides, anchor_stride):
    """utils.py:588-648: anchors [N, (y1, x1, y2, x2)] in pixels, level by level, (location, ratio) order."""
    out = []
    for i, scale in enumerate(scales):
        sc, ra = np.meshgrid(np.array([scale]), np.array(ratios))
        sc, ra = sc.flatten(), ra.flatten()
        heights = sc / np.sqrt(ra)
        widths = sc * np.sqrt(ra)
        sy = np.arange(0, feature_shapes[i][0], anchor_stride) * feature_strides[i]
        sx = np.arange(0, feature_shapes[i][1], anchor_stride) * feature_strides[i]
        sx, sy = np.meshgrid(sx, sy)
        bw, cx = np.meshgrid(widths, sx)
        bh, cy = np.meshgrid(heights, sy)
        centers = np.stack([cy, cx], axis=2).reshape([-1, 2])
        sizes = np.stack([bh, bw], axis=2).reshape([-1, 2])
        out.append(np.concatenate([centers - 0.5 * sizes, centers + 0.5 * sizes], axis=1))
    return np.concatenate(out, axis=0)


def norm_boxes(boxes, shape):
    """utils.py:858-872."""
    h, w = shape
    return np.divide(boxes - np.array([0, 0, 1, 1]), np.array([h - 1, w - 1, h - 1, w - 1])).astype(np.float32)


def apply_box_deltas(boxes: torch.Tensor, deltas: torch.Tensor) -> torch.Tensor:
    """model.py:219-240 apply_box_deltas_graph (f32)."""
    h = boxes[:, 2] - boxes[:, 0]
    w = boxes[:, 3] - boxes[:, 1]
    cy = boxes[:, 0] + 0.5 * h + deltas[:, 0] * h
    cx = boxes[:, 1] + 0.5 * w + deltas[:, 1] * w
    h = h * torch.exp(deltas[:, 2])
    w = w * torch.exp(deltas[:, 3])
    y1 = cy - 0.5 * h
    x1 = cx - 0.5 * w
    return torch.stack([y1, x1, y1 + h, x1 + w], dim=1)


def clip_boxes(boxes: torch.Tensor, window) -> torch.Tensor:
    """model.py:243-258 clip_boxes_graph; window (y1, x1, y2, x2)."""
    wy1, wx1, wy2, wx2 = window
    return torch.stack([boxes[:, 0].clamp(wy1, wy2), boxes[:, 1].clamp(wx1, wx2), boxes[:, 2].clamp(wy1, wy2),
                        boxes[:, 3].clamp(wx1, wx2)], dim=1)


# ---------------------------------------------------------------------------------- network
def _conv(cin, cout, k, stride=1, padding=0):
    return nn.Conv2d(cin, cout, k, stride=stride, padding=padding, bias=True)  # use_bias=True, BN folded


class _Bottleneck(nn.Module):
    """identity_block / conv_block (model.py:101-174); the inference BatchNorm is folded into the convs."""

    def __init__(self, cin, filters, stride, shortcut):
        super().__init__()
        f1, f2, f3 = filters
        self.a = _conv(cin, f1, 1, stride)
        self.b = _conv(f1, f2, 3, 1, 1)
        self.c = _conv(f2, f3, 1)
        self.sc = _conv(cin, f3, 1, stride) if shortcut else None

    def forward(self, x):
        y = F.relu(self.a(x))
        y = F.relu(self.b(y))
        y = self.c(y)
        return F.relu(y + (self.sc(x) if self.sc is not None else x))


class MaskRCNN(nn.Module):
    def __init__(self, config: Config | None = None, seed: int = 0, nms=None):
        super().__init__()
        self.config = cfg = config or Config()
        # the greedy NMS: the HIP kernels (nms_sorted); tests on a CPU pass the oracle's restatement
        self._nms = nms or nms_sorted
        assert cfg.BACKBONE in ("resnet50", "resnet101")
        self.conv1 = _conv(3, 64, 7, 2, 3)  # ZeroPadding2D(3) + 7x7 stride 2 (model.py:191-192)
        blocks = []
        cin = 64
        nid = {"resnet50": 5, "resnet101": 22}[cfg.BACKBONE]
        for stage, (filters, n, stride) in enumerate([((64, 64, 256), 2, 1), ((128, 128, 512), 3, 2),
                                                        ((256, 256, 1024), nid, 2), ((512, 512, 2048), 2, 2)]):
            st = [_Bottleneck(cin, filters, stride, True)]
            st += [_Bottleneck(filters[2], filters, 1, False) for _ in range(n)]
            blocks.append(nn.Sequential(*st))
            cin = filters[2]
        self.stages = nn.ModuleList(blocks)
        d = cfg.TOP_DOWN_PYRAMID_SIZE
        self.lat = nn.ModuleList([_conv(c, d, 1) for c in (256, 512, 1024, 2048)])  # fpn_c2p2 .. fpn_c5p5
        self.out = nn.ModuleList([_conv(d, d, 3, 1, 1) for _ in range(4)])           # fpn_p2 .. fpn_p5
        A = len(cfg.RPN_ANCHOR_RATIOS)
        self.rpn_shared = _conv(d, 512, 3, cfg.RPN_ANCHOR_STRIDE, 1)
        self.rpn_class = _conv(512, 2 * A, 1)
        self.rpn_bbox = _conv(512, 4 * A, 1)
        P, fc, nc = cfg.POOL_SIZE, cfg.FC_LAYERS_SIZE, cfg.NUM_CLASSES
        self.cls_conv1 = _conv(d, fc, P)  # mrcnn_class_conv1: 7x7 valid
        self.cls_conv2 = _conv(fc, fc, 1)
        self.cls_logits = nn.Linear(fc, nc)
        self.bbox_fc = nn.Linear(fc, nc * 4)
        self.mask_convs = nn.ModuleList([_conv(d, 256, 3, 1, 1) for _ in range(4)])
        self.mask_deconv = nn.ConvTranspose2d(256, 256, 2, stride=2)
        self.mask_out = _conv(256, nc, 1)
        self._init(seed)
        self._anchors = {}
        self._consts = {}

    @torch.no_grad()
    def _init(self, seed):
        """Seeded random weights (no checkpoint offline), He-normal; `calibrate` then scales every layer
        once on a seeded synthetic image (the role the reference's folded BatchNorm statistics play)."""
        g = torch.Generator().manual_seed(seed)
        self._seed = seed
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d, nn.Linear)):
                fan_in = m.weight[0].numel() if not isinstance(m, nn.ConvTranspose2d) else m.weight.shape[0] * 4
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * math.sqrt(2.0 / fan_in))
                m.bias.zero_()
        self._calibrated = False

    @torch.no_grad()
    def calibrate(self, device, image: torch.Tensor | None = None):
        """Layer-sequential unit-variance scaling in one forward pass over `image` (by default the first
        image `detect` sees; a seeded noise image when none is given) (every
        convolution's output rescaled to unit standard deviation as it is produced, the weights with it),
        then the residual branches' last convolutions at 0.2, the class logits scaled so that a few
        proposals per frame clear DETECTION_MIN_CONFIDENCE and the mask logits centred above the 0.5
        threshold: bounded activations through the 33 residual blocks, a realistic number of
        detections and masks per frame."""
        cfg = self.config
        S = cfg.IMAGE_MAX_DIM
        if image is None:
            g = torch.Generator().manual_seed(self._seed + 1)
            img = (torch.rand((S, S, 3), generator=g) * 255).to(torch.uint8).to(device)
        else:
            img = image.to(device)
        hooks = []

        def hook(mod, inp, out):
            sd = out.float().std().clamp(min=1e-6)
            mod.weight.div_(sd.to(mod.weight.dtype))
            mod.bias.div_(sd.to(mod.bias.dtype))
            return out / sd.to(out.dtype)

        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d, nn.Linear)):
                hooks.append(m.register_forward_hook(hook))
        self._calibrated = True
        try:
            self.detect(img)
        finally:
            for h in hooks:
                h.remove()
        for st in self.stages:
            for blk in st:
                blk.c.weight.mul_(0.2)
                blk.c.bias.mul_(0.2)
        # the class logits: a bias of 3 on six "object" classes, and the weights scaled so that about 2 %
        # of the calibration image's proposals clear DETECTION_MIN_CONFIDENCE (a few detections a frame)
        nc = cfg.NUM_CLASSES
        b = torch.zeros(nc, device=self.cls_logits.bias.device, dtype=self.cls_logits.bias.dtype)
        b[1:7] = 3.0
        self.cls_logits.bias.copy_(b)
        x, window, _ = self.mold(img)
        feats = self.backbone(x.to(cfg.DTYPE).contiguous(memory_format=torch.channels_last))
        lg, de = self.rpn(feats)
        rois = self.proposals(lg, de, self.anchors((S, S), img.device))
        pooled = self.roi_align(rois, feats[:4], cfg.POOL_SIZE, (S, S))
        sh = F.relu(self.cls_conv2(F.relu(self.cls_conv1(pooled)))).flatten(1)
        raw = (sh @ self.cls_logits.weight.t()).float()
        alpha = 1.0
        for a in [1.0 + 0.5 * k for k in range(60)]:
            p = torch.softmax(a * raw + b.float(), dim=1)
            sc, cl = p.max(dim=1)
            if ((sc >= cfg.DETECTION_MIN_CONFIDENCE) & (cl > 0)).float().mean().item() >= 0.02:
                alpha = a
                break
        self.cls_logits.weight.mul_(alpha)
        # mask logits centred at +2 (most of a box above the 0.5 threshold), so that detections reach the
        # dmask.py area rule (> 2000 px) and the fusion sees instances
        self.mask_out.bias.add_(2.0)
        # the refined boxes 3.5x the proposal's height and width (log-scale deltas over BBOX_STD_DEV): the
        # random RPN favours the smallest anchors (20x20 px at 640x480, profiles/r06/det/areas_probe.txt),
        # whose masks stay below the 2000-px rule and would leave the fusion without instances
        gb = torch.zeros(cfg.NUM_CLASSES, 4, device=self.bbox_fc.bias.device, dtype=torch.float32)
        gb[:, 2] = float(np.log(3.5)) / cfg.BBOX_STD_DEV[2]
        gb[:, 3] = float(np.log(3.5)) / cfg.BBOX_STD_DEV[3]
        self.bbox_fc.bias.add_(gb.view(-1).to(self.bbox_fc.bias.dtype))

    def _const(self, name, values, device):
        """Small constant tensors made once per device (no host-to-device copy inside a graph capture)."""
        key = (name, tuple(values), str(device))
        c = self._consts.get(key)
        if c is None:
            c = self._consts[key] = torch.tensor(values, dtype=torch.float32, device=device)
        return c

    # ---- stages of the graph
    def backbone(self, x):
        x = F.relu(self.conv1(x))
        # MaxPooling2D((3, 3), strides=2, padding="same"): TF pads the odd pixel at the bottom/right
        x = F.max_pool2d(F.pad(x, (0, 1, 0, 1), value=float("-inf")), 3, 2)
        cs = []
        for st in self.stages:
            x = st(x)
            cs.append(x)
        C2, C3, C4, C5 = cs
        P5 = self.lat[3](C5)
        P4 = F.interpolate(P5, scale_factor=2, mode="nearest") + self.lat[2](C4)
        P3 = F.interpolate(P4, scale_factor=2, mode="nearest") + self.lat[1](C3)
        P2 = F.interpolate(P3, scale_factor=2, mode="nearest") + self.lat[0](C2)
        P2, P3, P4, P5 = (self.out[i](p) for i, p in enumerate((P2, P3, P4, P5)))
        P6 = P5[:, :, ::2, ::2]  # MaxPooling2D(pool_size=1, strides=2)
        return [P2, P3, P4, P5, P6]

    def rpn(self, feats):
        logits, deltas = [], []
        for p in feats:
            s = F.relu(self.rpn_shared(p))
            # [1, C, H, W] -> NHWC -> [H * W * A, k]: the reference's reshape order (location, anchor)
            logits.append(self.rpn_class(s).permute(0, 2, 3, 1).reshape(-1, 2))
            deltas.append(self.rpn_bbox(s).permute(0, 2, 3, 1).reshape(-1, 4))
        return torch.cat(logits).float(), torch.cat(deltas).float()

    def anchors(self, image_shape, device):
        key = (tuple(image_shape), str(device))
        if key not in self._anchors:
            cfg = self.config
            shapes = [(int(math.ceil(image_shape[0] / s)), int(math.ceil(image_shape[1] / s))) for s in cfg.BACKBONE_STRIDES]
            a = generate_pyramid_anchors(cfg.RPN_ANCHOR_SCALES, cfg.RPN_ANCHOR_RATIOS, shapes, cfg.BACKBONE_STRIDES,
                                         cfg.RPN_ANCHOR_STRIDE)
            self._anchors[key] = torch.from_numpy(norm_boxes(a, image_shape[:2])).to(device)
        return self._anchors[key]

    def proposals(self, logits, deltas, anchors):
        """ProposalLayer (model.py:282-334)."""
        cfg = self.config
        scores = torch.softmax(logits, dim=1)[:, 1]
        k = min(cfg.PRE_NMS_LIMIT, scores.shape[0])
        top, ix = torch.topk(scores, k, sorted=True)
        d = deltas[ix] * self._const("rpn_std", cfg.RPN_BBOX_STD_DEV, deltas.device)
        boxes = clip_boxes(apply_box_deltas(anchors[ix], d), (0.0, 0.0, 1.0, 1.0))
        keep, count = self._nms(boxes, cfg.RPN_NMS_THRESHOLD, cfg.POST_NMS_ROIS_INFERENCE)
        valid = keep >= 0
        rois = torch.where(valid[:, None], boxes[keep.clamp(min=0).long()], torch.zeros((), device=boxes.device))
        return rois  # [POST_NMS_ROIS_INFERENCE, 4], zero-padded (tf.pad)

    def roi_align(self, rois, feats, pool, image_shape):
        """PyramidROIAlign (model.py:374-452): level by box size, tf.image.crop_and_resize per level,
        the pooled crops back in the rois' order.  [n, C, pool, pool]."""
        h = rois[:, 2] - rois[:, 0]
        w = rois[:, 3] - rois[:, 1]
        area = float(image_shape[0] * image_shape[1])
        lvl = torch.log2(torch.sqrt(h * w) / (224.0 / math.sqrt(area)))
        lvl = torch.clamp(4 + torch.round(lvl), 2, 5)  # empty (zero) rois: log2(0) = -inf -> level 2
        lvl = torch.where(torch.isnan(lvl), torch.full_like(lvl, 2.0), lvl).long()
        if rois.device.type == "cuda" and feats[0].dtype in (torch.float16, torch.bfloat16) and ROI_ALIGN_HIP:
            return roi_align_dev(rois, lvl, feats, pool)
        n, Cn = rois.shape[0], feats[0].shape[1]
        out = torch.zeros((n, Cn, pool, pool), dtype=feats[0].dtype, device=rois.device)
        i = torch.arange(pool, device=rois.device, dtype=torch.float32)
        for L in range(2, 6):
            fm = feats[L - 2]
            H, W = fm.shape[2], fm.shape[3]
            # every roi sampled on every level and the level's samples kept (static shapes: no host
            # synchronisation, so a whole detect() can be captured in a HIP graph)
            b = rois
            # crop_and_resize sample positions: y = y1 (H - 1) + i (y2 - y1) (H - 1) / (pool - 1)
            ys = b[:, 0:1] * (H - 1) + i[None, :] * ((b[:, 2:3] - b[:, 0:1]) * (H - 1) / (pool - 1))
            xs = b[:, 1:2] * (W - 1) + i[None, :] * ((b[:, 3:4] - b[:, 1:2]) * (W - 1) / (pool - 1))
            gy = ys / (H - 1) * 2 - 1
            gx = xs / (W - 1) * 2 - 1
            grid = torch.stack([gx[:, None, :].expand(-1, pool, -1), gy[:, :, None].expand(-1, -1, pool)], dim=-1)
            # one batch: every roi's pool x pool samples as rows of a single grid over the level's map
            smp = F.grid_sample(fm.float(), grid.reshape(1, n * pool, pool, 2), mode="bilinear",
                                padding_mode="zeros", align_corners=True)  # [1, C, n pool, pool]
            smp = smp.view(Cn, n, pool, pool).permute(1, 0, 2, 3)
            inside = ((ys >= 0) & (ys <= H - 1))[:, :, None] & ((xs >= 0) & (xs <= W - 1))[:, None, :]
            keep = inside[:, None] & (lvl == L)[:, None, None, None]
            out = out + torch.where(keep, smp, torch.zeros((), device=smp.device)).to(out.dtype)
        return out

    def classifier(self, pooled):
        x = F.relu(self.cls_conv1(pooled))
        x = F.relu(self.cls_conv2(x)).flatten(1)
        logits = self.cls_logits(x).float()
        deltas = self.bbox_fc(x).float().view(-1, self.config.NUM_CLASSES, 4)
        return torch.softmax(logits, dim=1), deltas

    def detections(self, rois, probs, deltas, window):
        """refine_detections_graph (model.py:689-784): [n, (y1, x1, y2, x2, class_id, score)], the
        per-class NMS as one NMS over class-offset boxes (boxes of different classes never overlap)."""
        cfg = self.config
        score, cls = probs.max(dim=1)
        d = deltas[torch.arange(deltas.shape[0], device=deltas.device), cls] * self._const("bbox_std", cfg.BBOX_STD_DEV,
                                                                                           deltas.device)
        refined = clip_boxes(apply_box_deltas(rois, d), window)
        ok = (cls > 0) & (score >= cfg.DETECTION_MIN_CONFIDENCE) & (rois.abs().sum(1) > 0)
        score_k = torch.where(ok, score, torch.full_like(score, -1.0))
        order = torch.argsort(score_k, descending=True, stable=True)
        off = refined[order] + (cls[order].float() * 2.0)[:, None]
        n_ok = ok.sum()
        keep, count = self._nms(off, cfg.DETECTION_NMS_THRESHOLD, cfg.DETECTION_MAX_INSTANCES)
        # boxes past n_ok (not candidates) sort last and are cut by their -1 score below
        k = keep.clamp(min=0).long()
        sel = order[k]
        valid = (keep >= 0) & (keep < n_ok)  # kept positions among the candidates (they sort first)
        det = torch.cat([refined[sel], cls[sel].float()[:, None], score[sel][:, None]], dim=1)
        return det * valid[:, None].float()  # zero rows past the detections (tf.pad)

    def mask_head(self, pooled):
        x = pooled
        for c in self.mask_convs:
            x = F.relu(c(x))
        x = F.relu(self.mask_deconv(x))
        return torch.sigmoid(self.mask_out(x).float())  # [n, classes, 28, 28]

    # ---- the reference's detect(): mold, run, unmold
    def mold(self, image_u8: torch.Tensor):
        """mold_inputs (model.py:2332-2368) for one HxWx3 u8 device image: square resize + padding,
        minus MEAN_PIXEL; returns (molded NCHW, window (y1, x1, y2, x2) pixels, scale)."""
        cfg = self.config
        h, w = image_u8.shape[:2]
        scale = max(1.0, cfg.IMAGE_MIN_DIM / min(h, w))
        if round(max(h, w) * scale) > cfg.IMAGE_MAX_DIM:
            scale = cfg.IMAGE_MAX_DIM / max(h, w)
        nh, nw = round(h * scale), round(w * scale)
        x = image_u8.permute(2, 0, 1)[None].float()
        if scale != 1:
            x = F.interpolate(x, size=(nh, nw), mode="bilinear", align_corners=False)
        top, left = (cfg.IMAGE_MAX_DIM - nh) // 2, (cfg.IMAGE_MAX_DIM - nw) // 2
        x = x - self._const("mean", cfg.MEAN_PIXEL, x.device)[None, :, None, None]
        x = F.pad(x, (left, cfg.IMAGE_MAX_DIM - nw - left, top, cfg.IMAGE_MAX_DIM - nh - top))
        return x, (top, left, nh + top, nw + left), scale

    @torch.no_grad()
    def detect(self, image_u8: torch.Tensor, compact: bool = True) -> dict:
        """One HxWx3 u8 RGB image on the device -> {rois [N, 4] int32 pixels, class_ids [N], scores [N],
        masks [H, W, N] u8}, all device tensors (model.py:2436-2492 for one image).  compact=False: no
        host synchronisation -- N = DETECTION_MAX_INSTANCES rows, the rows past the detections (and
        those unmold_detections drops for zero area) with class 0 and an empty mask, which the dmask.py
        rule (semtsdf_masks_to_labels, areas > 2000) never keeps: for a producer stream."""
        cfg = self.config
        dev = image_u8.device
        if not self._calibrated:
            self.calibrate(dev, image_u8)
        H0, W0 = int(image_u8.shape[0]), int(image_u8.shape[1])
        x, window, _ = self.mold(image_u8)
        shape = (cfg.IMAGE_MAX_DIM, cfg.IMAGE_MAX_DIM)
        x = x.to(cfg.DTYPE).contiguous(memory_format=torch.channels_last if CHANNELS_LAST else torch.contiguous_format)
        feats = self.backbone(x)
        logits, deltas = self.rpn(feats)
        rois = self.proposals(logits, deltas, self.anchors(shape, dev))
        mfeats = feats[:4]
        probs, bdeltas = self.classifier(self.roi_align(rois, mfeats, cfg.POOL_SIZE, shape))
        nwin = norm_boxes(np.array(window, dtype=np.float64), shape)
        det = self.detections(rois, probs, bdeltas, tuple(float(v) for v in nwin))
        masks = self.mask_head(self.roi_align(det[:, :4], mfeats, cfg.MASK_POOL_SIZE, shape))
        return self.unmold(det, masks, (H0, W0), shape, nwin, compact)

    def unmold(self, det, masks, orig_shape, image_shape, nwin, compact=True):
        """unmold_detections (model.py:2371-2433) + unmold_mask (utils.py:565-586), on the device:
        the detections (class id > 0) in pixels of the original image and their masks pasted at the
        boxes (bilinear resize of the 28x28 mask, >= 0.5)."""
        H0, W0 = orig_shape
        dev = det.device
        # detections come first, zero rows after them
        n = int((det[:, 4] > 0).sum().item()) if compact else int(det.shape[0])
        d = det[:n]
        wy1, wx1, wy2, wx2 = (float(v) for v in nwin)
        shift = self._const("shift", (wy1, wx1, wy1, wx1), dev)
        scale = self._const("scale", (wy2 - wy1, wx2 - wx1, wy2 - wy1, wx2 - wx1), dev)
        b = (d[:, :4] - shift) / scale
        px = torch.round(b * self._const("den", (H0 - 1, W0 - 1, H0 - 1, W0 - 1), dev)
                         + self._const("den_shift", (0, 0, 1, 1), dev)).to(torch.int32)
        cls = d[:, 4].long()
        ok = ((px[:, 2] - px[:, 0]) * (px[:, 3] - px[:, 1]) > 0) & (cls > 0)
        if compact:
            px, cls, scores = px[ok], cls[ok], d[ok, 5]
            m = masks[:n][ok]
        else:  # fixed rows: the dropped ones keep class 0 and get an empty box (and mask) below
            px = px * ok[:, None].to(px.dtype)
            cls = cls * ok.long()
            scores = d[:, 5] * ok.float()
            m = masks[:n]
        m = m[torch.arange(m.shape[0], device=dev), cls]  # [N, 28, 28] of each detection's class
        N = int(px.shape[0])
        if N == 0:
            return {"rois": px, "class_ids": cls.to(torch.int32), "scores": scores,
                    "masks": torch.zeros((H0, W0, 0), dtype=torch.uint8, device=dev)}
        # output pixel (y, x) of box (y1, x1, y2, x2) samples the mask at ((y - y1 + 0.5) 28 / h - 0.5),
        # i.e. grid coordinate (2 (y - y1) + 1) / h - 1 with align_corners=False; outside the box: 0
        ys = torch.arange(H0, device=dev, dtype=torch.float32)
        xs = torch.arange(W0, device=dev, dtype=torch.float32)
        y1, x1, y2, x2 = (px[:, k].float()[:, None] for k in range(4))
        # (the empty rows of the fixed-row form have zero extents: a unit divisor keeps their grid
        # finite; `inside` below zeroes them)
        gy = (2 * (ys[None] - y1) + 1) / (y2 - y1).clamp(min=1.0) - 1  # [N, H0]
        gx = (2 * (xs[None] - x1) + 1) / (x2 - x1).clamp(min=1.0) - 1  # [N, W0]
        grid = torch.stack([gx[:, None, :].expand(-1, H0, -1), gy[:, :, None].expand(-1, -1, W0)], dim=-1)
        full = F.grid_sample(m[:, None], grid, mode="bilinear", padding_mode="zeros", align_corners=False)[:, 0]
        inside = ((ys[None] >= y1) & (ys[None] < y2))[:, :, None] & ((xs[None] >= x1) & (xs[None] < x2))[:, None, :]
        full = ((full >= 0.5) & inside).to(torch.uint8)
        return {"rois": px, "class_ids": cls.to(torch.int32), "scores": scores,
                "masks": full.permute(1, 2, 0).contiguous()}


class GraphDetector:
    """`MaskRCNN.detect(compact=False)` for one image size captured in a HIP graph (torch.cuda.CUDAGraph:
    the backbone's and heads' several hundred launches, the NMS kernels and the unmold replayed as one):
    a frame is one copy into the static input and one replay on the current stream; the returned tensors
    are static and are overwritten by the next call.  Calibrate the model first (detect() would do it
    inside the capture otherwise)."""

    def __init__(self, model: MaskRCNN, image_shape, device, warmup: int = 3):
        if not model._calibrated:
            raise RuntimeError("calibrate the model before capturing it")
        self.model = model
        self.inp = torch.zeros(tuple(image_shape), dtype=torch.uint8, device=device)
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(warmup):  # MIOpen's solver choice and the allocator's pools settle first
                model.detect(self.inp, compact=False)
        torch.cuda.current_stream(device).wait_stream(side)
        torch.cuda.synchronize(device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = model.detect(self.inp, compact=False)

    def __call__(self, image_u8: torch.Tensor) -> dict:
        self.inp.copy_(image_u8)
        self.graph.replay()
        return self.out
