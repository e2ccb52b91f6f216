"""mmcv DropPath restatement; the per-sample keep mask can be injected for goldens."""
import torch
import torch.nn as nn

# When not None: a list that DropPath pops per-call masks [B] (values 0/1) from.
INJECTED_MASKS = None


class DropPath(nn.Module):
    def __init__(self, drop_prob=0.1):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        keep = 1.0 - self.drop_prob
        shape = (x.shape[0],) + (1,) * (x.ndim - 1)
        if INJECTED_MASKS is not None:
            mask = INJECTED_MASKS.pop(0).to(x.dtype).reshape(shape)
        else:
            mask = (keep + torch.rand(shape, dtype=x.dtype, device=x.device)).floor()
        return x.div(keep) * mask


def build_dropout(cfg):
    cfg = dict(cfg)
    assert cfg.pop("type") == "DropPath"
    return DropPath(**cfg)


class FFN(nn.Module):  # imported by the reference, never used on the hot path
    pass
