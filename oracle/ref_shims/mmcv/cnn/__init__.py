"""mmcv.cnn restatement: build_norm_layer and ConvModule (conv -> norm -> act)."""
import torch.nn as nn

_NORM = {"BN": nn.BatchNorm2d, "BN2d": nn.BatchNorm2d,
         # single-process CPU goldens: SyncBN has BatchNorm2d semantics
         "SyncBN": nn.BatchNorm2d}


def build_norm_layer(cfg, num_features, postfix=""):
    cfg = dict(cfg)
    layer_type = cfg.pop("type")
    requires_grad = cfg.pop("requires_grad", True)
    cfg.setdefault("eps", 1e-5)
    layer = _NORM[layer_type](num_features, **cfg)
    for p in layer.parameters():
        p.requires_grad = requires_grad
    return "bn" + str(postfix), layer


class ConvModule(nn.Module):
    """conv (bias only when there is no norm) -> norm ('bn') -> activate (ReLU)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 dilation=1, groups=1, bias="auto", conv_cfg=None, norm_cfg=None,
                 act_cfg=dict(type="ReLU"), inplace=True, **kwargs):
        super().__init__()
        self.with_norm = norm_cfg is not None
        self.with_activation = act_cfg is not None
        if bias == "auto":
            bias = not self.with_norm
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding,
                              dilation, groups, bias=bias)
        if self.with_norm:
            self.norm_name, norm = build_norm_layer(norm_cfg, out_channels)
            self.add_module(self.norm_name, norm)
        if self.with_activation:
            assert act_cfg["type"] == "ReLU"
            self.activate = nn.ReLU(inplace=inplace)

    def forward(self, x):
        x = self.conv(x)
        if self.with_norm:
            x = getattr(self, self.norm_name)(x)
        if self.with_activation:
            x = self.activate(x)
        return x
