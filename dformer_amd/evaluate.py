"""Multi-scale + flip evaluation and mIoU metrics on the HIP path.

Mirrors the reference's `utils/val_mm.py:325-472 evaluate_msf` and `utils/metrics_new.py:6-47
Metrics` (same names, arguments and results). Per batch and scale s the inputs are resized to
ceil(s*H/32)*32 x ceil(s*W/32)*32 (bilinear, align_corners=True) [and flipped], the model runs its
eval forward (ham head: 7 NMF steps), and one kernel folds the model's own logits upsampling
(align_corners=False), the flip back, the resize to the label size (align_corners=True), the
softmax and the accumulation over scales into a float32 [B*H*W, ncls] buffer; the confusion
histogram is another kernel. Sliding-window inference (`slide_inference`) and prediction PNG
export (`save_dir`) are not on the path and raise.
"""
import math

import torch

from . import kernels as K
from .decoders import _nhwc_rows


class Metrics:
    """utils/metrics_new.py:6-47: confusion histogram over labelled pixels, IoU / F1 / accuracy."""

    def __init__(self, num_classes, ignore_label, device):
        self.ignore_label = ignore_label
        self.num_classes = num_classes
        self._hist = torch.zeros(num_classes * num_classes, dtype=torch.int64, device=device)
        self.index = 0

    @property
    def hist(self):
        return self._hist.view(self.num_classes, self.num_classes).float()

    def update_hist(self, hist):
        self._hist += hist.to(self._hist.device).reshape(-1).round().long()

    def update_rows(self, acc, target):
        """acc: float32 [B*H*W, ncls] class scores (NHWC rows), target: [B, H, W] labels."""
        self.index += 1
        K.seg_confusion(acc, target.long().contiguous(), self.num_classes, self.ignore_label, self._hist)

    def update(self, pred, target):
        """pred: [B, ncls, H, W] class scores (any layout), target: [B, H, W]."""
        rows = pred.float().permute(0, 2, 3, 1).contiguous().view(-1, pred.shape[1])
        self.update_rows(rows, target)

    def compute_iou(self):
        h = self.hist
        ious = h.diag() / (h.sum(0) + h.sum(1) - h.diag())
        ious[ious.isnan()] = 0.0
        miou = ious.mean().item()
        ious *= 100
        miou *= 100
        return ious.cpu().numpy().round(2).tolist(), round(miou, 2)

    def compute_f1(self):
        h = self.hist
        f1 = 2 * h.diag() / (h.sum(0) + h.sum(1))
        f1[f1.isnan()] = 0.0
        mf1 = f1.mean().item()
        f1 *= 100
        mf1 *= 100
        return f1.cpu().numpy().round(2).tolist(), round(mf1, 2)

    def compute_pixel_acc(self):
        h = self.hist
        acc = h.diag() / h.sum(1)
        acc[acc.isnan()] = 0.0
        macc = acc.mean().item()
        acc *= 100
        macc *= 100
        return acc.cpu().numpy().round(2).tolist(), round(macc, 2)


def msf_size(H, W, scale):
    """val_mm.py:359-364: the scaled input size, rounded up to a multiple of 32."""
    nh, nw = int(scale * H), int(scale * W)
    return int(math.ceil(nh / 32)) * 32, int(math.ceil(nw / 32)) * 32


@torch.no_grad()
def msf_scores(model, rgb, modal_x, num_classes, scales, flip, out_shape=None):
    """Summed softmax scores over scales (and flips) of one batch: float32 [B*H*W, ncls] rows
    (val_mm.py:355-392 for one batch; `scaled_logits` of the reference, channels last). Like the
    reference (val_mm.py:355-356) the scaled sizes and the score buffer follow the LABEL's
    (B, H, W) = out_shape (default: the image's own size)."""
    B, H, W = out_shape if out_shape is not None else (rgb.shape[0], rgb.shape[2], rgb.shape[3])
    if rgb.shape[0] != B or modal_x.shape[0] != B:
        raise ValueError(f"msf_scores: batch of the images {rgb.shape[0]} != labels {B}")
    acc = torch.zeros(B * H * W, num_classes, device=rgb.device, dtype=torch.float32)
    for scale in scales:
        size = msf_size(H, W, scale)
        for f in ((False, True) if flip else (False,)):
            x = K.resize_nchw(rgb, size, True, flip=f)
            e = K.resize_nchw(modal_x, size, True, flip=f)
            low = model._low_logits(x, e)
            rows, (b, h, w) = _nhwc_rows(low)
            K.msf_accumulate(rows, b, h, w, num_classes, size, (H, W), f, acc)
    return acc


@torch.no_grad()
def evaluate_msf(model, dataloader, config, device, scales, flip, engine=None, save_dir=None, sliding=False):
    """val_mm.py:325-472. dataloader yields dicts with 'rgb', 'modal_x', 'gt'. Returns the Metrics
    (a list of every rank's Metrics when engine.distributed, like the reference)."""
    if sliding:
        raise NotImplementedError("evaluate_msf: slide_inference is outside the hot path (SURVEY.md §2)")
    if save_dir is not None:
        raise NotImplementedError("evaluate_msf: prediction image export is outside the hot path (SURVEY.md §2)")
    model.eval()
    metrics = Metrics(config.num_classes, config.background, device)
    for batch in dataloader:
        rgb = batch["rgb"].to(device)
        modal_x = batch["modal_x"].to(device)
        gt = batch["gt"].to(device)
        acc = msf_scores(model, rgb, modal_x, config.num_classes, scales, flip, out_shape=tuple(gt.shape))
        metrics.update_rows(acc, gt)
    if engine is not None and getattr(engine, "distributed", False):
        all_metrics = [None for _ in range(engine.world_size)]
        torch.distributed.all_gather_object(all_metrics, metrics)
        return all_metrics
    return metrics
