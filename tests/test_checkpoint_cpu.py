"""Checkpoint I/O and optimizer-state compatibility with the reference's files (CPU).

The reference saves {"model", "optimizer" (torch.optim.AdamW over group_weight's two groups),
"epoch", "iteration"} (utils/engine/engine.py:101-126) and loads pretrained backbones from
`state_dict_ema` / `state_dict` with `backbone.` / `module.` stripped (DFormer.py:254-276). These
tests build such files with plain torch (a real torch.optim.AdamW run) and check that
dformer_amd reads and writes them faithfully.
"""
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dformer_amd import checkpoint as ckpt  # noqa: E402
from dformer_amd.train import FusedAdamW, group_weight  # noqa: E402


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3, padding=1)
        self.bn = nn.BatchNorm2d(8)
        self.fc = nn.Linear(8, 6)
        self.ln = nn.LayerNorm(6)
        self.unused = nn.Linear(2, 2)
        self.unused.weight.requires_grad_(False)
        self.unused.bias.requires_grad_(False)

    def forward(self, x):
        return self.ln(self.fc(torch.relu(self.bn(self.conv(x))).mean(dim=(2, 3))))


def _torch_adamw_run(net, steps=2):
    decay, no_decay = group_weight(net)
    opt = torch.optim.AdamW([dict(params=decay, lr=6e-5), dict(params=no_decay, weight_decay=0.0, lr=6e-5)],
                            lr=6e-5, betas=(0.9, 0.999), weight_decay=0.01)
    for s in range(steps):
        opt.zero_grad()
        net(torch.randn(2, 3, 5, 5, generator=torch.Generator().manual_seed(s))).square().mean().backward()
        opt.step()
    return opt


def test_optimizer_state_roundtrip_with_torch_adamw():
    torch.manual_seed(0)
    ref = _Net()
    topt = _torch_adamw_run(ref)
    tsd = topt.state_dict()
    net = _Net()
    net.load_state_dict(ref.state_dict())
    opt = FusedAdamW(net, compute_dtype=torch.float32)
    opt.load_state_dict(tsd)
    assert opt.step_count == 2
    names = {id(p): n for n, p in net.named_parameters()}
    rnames = dict(ref.named_parameters())
    idx = 0
    for plist, g in zip(opt.full_groups, opt.groups):
        for p in plist:
            if p in g.slots:
                off, k = g.slots[p]
                st = tsd["state"][idx]
                assert torch.equal(g.m[off:off + k], st["exp_avg"].reshape(-1)), names[id(p)]
                assert torch.equal(g.v[off:off + k], st["exp_avg_sq"].reshape(-1))
            else:
                assert idx not in tsd["state"] and not rnames[names[id(p)]].requires_grad
            idx += 1
    ours = opt.state_dict()
    assert set(ours["state"]) == set(tsd["state"])
    for i, st in tsd["state"].items():
        assert torch.equal(ours["state"][i]["exp_avg"], st["exp_avg"])
        assert torch.equal(ours["state"][i]["exp_avg_sq"], st["exp_avg_sq"])
        assert float(ours["state"][i]["step"]) == float(st["step"])
    for a, b in zip(ours["param_groups"], tsd["param_groups"]):
        assert a["params"] == b["params"] and a["weight_decay"] == b["weight_decay"]
        assert set(a) == set(b)
    # and torch can consume ours
    ref2 = _Net()
    decay, no_decay = group_weight(ref2)
    topt2 = torch.optim.AdamW([dict(params=decay), dict(params=no_decay, weight_decay=0.0)], lr=6e-5)
    topt2.load_state_dict(ours)


def test_save_restore_checkpoint_segmentor(tmp_path):
    import bench
    from dformer_amd.segmentor import EncoderDecoder
    torch.manual_seed(1)
    m1 = EncoderDecoder(cfg=bench.make_cfg("DFormer-Tiny", "ham"))
    o1 = FusedAdamW(m1, compute_dtype=torch.float32)
    for g in o1.groups:  # pretend some optimisation happened
        g.m.uniform_()
        g.v.uniform_()
    o1.step_count = 7
    path = str(tmp_path / "epoch-3.pth")
    ckpt.save_checkpoint(path, m1, o1, epoch=3, iteration=1234)
    raw = torch.load(path, weights_only=True)
    assert set(raw) == {"model", "optimizer", "epoch", "iteration"}
    assert not any(k.startswith("module.") for k in raw["model"])

    torch.manual_seed(2)
    m2 = EncoderDecoder(cfg=bench.make_cfg("DFormer-Tiny", "ham"))
    o2 = FusedAdamW(m2, compute_dtype=torch.float32)
    epoch, it = ckpt.restore_checkpoint(path, m2, o2)
    assert (epoch, it) == (4, 1234) and o2.step_count == 7
    for (k, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    for g1, g2 in zip(o1.groups, o2.groups):
        assert torch.equal(g1.flat, g2.flat) and torch.equal(g1.m, g2.m) and torch.equal(g1.v, g2.v)


def test_load_model_accepts_reference_layouts(tmp_path):
    import bench
    from dformer_amd.segmentor import EncoderDecoder
    torch.manual_seed(3)
    src = EncoderDecoder(cfg=bench.make_cfg("DFormer-Tiny", "ham"))
    sd = src.state_dict()
    for wrap in ("model", "state_dict", "module", None):
        body = {"module." + k: v for k, v in sd.items()} if wrap == "module" else sd
        obj = {wrap: body} if wrap else body
        p = str(tmp_path / f"{wrap}.pth")
        torch.save(obj, p)
        dst = EncoderDecoder(cfg=bench.make_cfg("DFormer-Tiny", "ham"))
        ckpt.load_model(dst, p)
        for k, v in dst.state_dict().items():
            assert torch.equal(v, sd[k]), (wrap, k)


def test_pretrained_backbone_prefixes_and_freeze(tmp_path):
    from dformer_amd.encoder import DFormer_Tiny
    torch.manual_seed(4)
    src = DFormer_Tiny()
    part = {k: v for k, v in src.state_dict().items() if k.startswith(("downsample_layers.", "stages.0."))}
    for key, prefix in (("state_dict_ema", "backbone."), ("state_dict", "module.")):
        p = str(tmp_path / f"{key}.pth")
        torch.save({key: {prefix + k: v for k, v in part.items()}, "other": {}}, p)
        dst = DFormer_Tiny()
        missing, unexpected = ckpt.load_pretrained_backbone(dst, p)
        assert not unexpected
        dsd = dst.state_dict()
        for k, v in part.items():
            assert torch.equal(dsd[k], v), k
        for n, prm in dst.named_parameters():
            loaded = any(n == k or n.startswith(k + ".") for k in part)
            assert prm.requires_grad == (not loaded) or "stem_e_fc" in n, n


def test_freeze_after_optimizer_is_rejected():
    """load_pretrained_backbone(freeze=True) must not silently leave frozen parameters inside a live
    FusedAdamW (the reference freezes in the constructor, before the optimizer exists)."""
    import pytest
    torch.manual_seed(0)
    net = _Net()
    opt = FusedAdamW(net, compute_dtype=torch.float32)
    with pytest.raises(RuntimeError, match="after FusedAdamW"):
        ckpt.load_pretrained_backbone(net, {"state_dict": {k: v.clone() for k, v in net.state_dict().items()}})
    assert all(p.requires_grad for p in (net.fc.weight, net.conv.weight))
    del opt
    net2 = _Net()  # load + freeze first, then build the optimizer: fine
    ckpt.load_pretrained_backbone(net2, {"state_dict": {k: v.clone() for k, v in net.state_dict().items()}})
    assert not net2.fc.weight.requires_grad


def test_segmentor_rejects_unsupported_criterion():
    import pytest
    import bench
    from dformer_amd.segmentor import EncoderDecoder
    cfg = bench.make_cfg("DFormer-Tiny", "ham")
    EncoderDecoder(cfg=cfg, criterion=nn.CrossEntropyLoss(reduction="none", ignore_index=255))
    for bad in (nn.CrossEntropyLoss(weight=torch.ones(40), reduction="none", ignore_index=255),
                nn.CrossEntropyLoss(reduction="mean", ignore_index=255),
                nn.CrossEntropyLoss(reduction="none", ignore_index=0),
                nn.CrossEntropyLoss(reduction="none", ignore_index=255, label_smoothing=0.1)):
        with pytest.raises(NotImplementedError):
            EncoderDecoder(cfg=cfg, criterion=bad)
