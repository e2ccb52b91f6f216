"""EncoderDecoder (models/builder.py:91-235): backbone + decode head + CE loss, on HIP kernels.

forward(rgb, modal_x, label) -> (loss, out) in training, out in eval, like the reference. The
backbone's `(outs, None)` tuple is indexed before the decode head (the reference HEAD passes the
tuple through and crashes, SURVEY.md §3.0 #2 — the intended upstream semantics are reproduced).
`out` is the full-resolution logits (bilinear, align_corners=False); during training it is only
materialised when `return_logits` is True (the loss itself is fused and never needs it).
"""
import torch
import torch.nn as nn

from . import kernels as K
from .decoders import DecoderHead, LightHamHead, SegLossFn, _nhwc_rows
from .encoder import DFormer_Base, DFormer_Large, DFormer_Small, DFormer_Tiny
from .functional import invalidate_weights

BACKBONES = {"DFormer-Tiny": (DFormer_Tiny, [32, 64, 128, 256]), "DFormer-Small": (DFormer_Small, [64, 128, 256, 512]),
             "DFormer-Base": (DFormer_Base, [64, 128, 256, 512]), "DFormer-Large": (DFormer_Large, [96, 192, 288, 576])}


def _check_criterion(criterion, ignore_index):
    """The loss is the fused kernel of builder.py:203,230: unweighted CrossEntropyLoss(reduction='none',
    ignore_index=cfg.background) followed by the mean over valid pixels (what train.py:189-194
    passes). Anything else would be silently ignored, so it is rejected."""
    if criterion is None:
        return
    ok = (isinstance(criterion, nn.CrossEntropyLoss) and criterion.weight is None and
          criterion.reduction == "none" and criterion.ignore_index == ignore_index and
          float(getattr(criterion, "label_smoothing", 0.0)) == 0.0)
    if not ok:
        raise NotImplementedError(
            f"EncoderDecoder: the fused segmentation loss implements CrossEntropyLoss(reduction='none', "
            f"ignore_index={ignore_index}) without class weights or label smoothing (utils/train.py:189-194); "
            f"got {criterion!r}")


class EncoderDecoder(nn.Module):
    def __init__(self, cfg=None, criterion=None, norm_layer=nn.BatchNorm2d, syncbn=False):
        super().__init__()
        self.cfg = cfg
        self.norm_layer = norm_layer
        backbone, self.channels = BACKBONES[cfg.backbone]
        norm_cfg = dict(type="SyncBN" if syncbn else "BN", requires_grad=True)
        dpr = cfg.drop_path_rate if getattr(cfg, "drop_path_rate", None) is not None else 0.1
        self.encoder_backbone = backbone(drop_path_rate=dpr, norm_cfg=norm_cfg)
        bn_eps = getattr(cfg, "bn_eps", 1e-3)
        bn_mom = getattr(cfg, "bn_momentum", 0.1)
        if cfg.decoder == "MLPDecoder":
            self.decode_head = DecoderHead(in_channels=self.channels, num_classes=cfg.num_classes,
                                           norm_layer=norm_layer, embed_dim=cfg.decoder_embed_dim, bn_eps=bn_eps,
                                           bn_momentum=bn_mom, syncbn=syncbn)
        elif cfg.decoder == "ham":
            self.decode_head = LightHamHead(in_channels=self.channels[1:], num_classes=cfg.num_classes,
                                            in_index=[1, 2, 3], norm_cfg=norm_cfg, channels=cfg.decoder_embed_dim,
                                            bn_eps=bn_eps, bn_momentum=bn_mom)
        else:
            raise NotImplementedError(f"decoder {cfg.decoder!r} is outside the hot path (SURVEY.md §2)")
        self.aux_head = None
        _check_criterion(criterion, getattr(cfg, "background", 255))
        self.criterion = criterion
        self.ignore_index = getattr(cfg, "background", 255)
        self.return_logits = True

    def set_compute_dtype(self, dtype):
        self.encoder_backbone.compute_dtype = dtype
        return self

    def load_state_dict(self, *a, **k):
        r = super().load_state_dict(*a, **k)
        invalidate_weights()
        return r

    def _low_logits(self, rgb, modal_x):
        outs = self.encoder_backbone(rgb, modal_x)[0]
        K.TAG = "decoder"
        return self.decode_head.forward(outs)

    def _upsample(self, low, size):
        rows, (B, h, w) = _nhwc_rows(low)
        up = K.bilinear(rows.contiguous(), (h, w), tuple(size), B)
        return up.view(B, size[0], size[1], -1).permute(0, 3, 1, 2)

    def encode_decode(self, rgb, modal_x):
        low = self._low_logits(rgb, modal_x)
        return self._upsample(low, rgb.shape[-2:])

    def forward(self, rgb, modal_x=None, label=None):
        low = self._low_logits(rgb, modal_x)
        if label is None:
            return self._upsample(low, rgb.shape[-2:])
        rows, (B, h, w) = _nhwc_rows(low)
        K.TAG = "loss"
        loss = SegLossFn.apply(rows.contiguous(), B, h, w, label.long(), self.ignore_index)
        out = self._upsample(low.detach(), rgb.shape[-2:]) if self.return_logits else low
        return loss, out
