"""Checkpoint I/O compatible with the reference's files.

  load_pretrained_backbone   DFormer.init_weights (models/encoders/DFormer.py:254-276): a
                             `state_dict_ema` or `state_dict` entry, `backbone.` / `module.` prefixes
                             stripped, non-strict load, and — as the reference does — every loaded
                             backbone parameter frozen (requires_grad = False).
  load_model                 utils/pyt_utils.py:155-191: `model` / `state_dict` / `module` entry,
                             strict load (a `module.` prefix from a DDP save is stripped: this
                             framework never wraps the model in DDP).
  save_checkpoint            utils/engine/engine.py:101-126: {"model", "optimizer", "epoch", "iteration"}
                             with `module.` stripped and the optimizer in torch.optim.AdamW format.
  restore_checkpoint         utils/engine/engine.py:161-182 (epoch + 1, iteration as saved).

Files are read with torch.load(weights_only=True): nothing in a checkpoint is executed.
"""
from collections import OrderedDict

import torch

from .functional import has_grad_slot, invalidate_weights


def _read(src):
    if isinstance(src, (str, bytes)) or hasattr(src, "read"):
        return torch.load(src, map_location="cpu", weights_only=True)
    return src


def _strip(sd, prefix):
    return OrderedDict((k[len(prefix):] if k.startswith(prefix) else k, v) for k, v in sd.items())


def load_pretrained_backbone(backbone, src, freeze=True):
    """Returns (missing, unexpected) key lists like mmcv's non-strict load."""
    raw = _read(src)
    sd = raw["state_dict_ema"] if "state_dict_ema" in raw else raw.get("state_dict", raw)
    sd = _strip(sd, "backbone.")
    if next(iter(sd), "").startswith("module."):
        sd = _strip(sd, "module.")
    if freeze:
        keys = set(sd)
        to_freeze = [(name, p) for name, p in backbone.named_parameters()
                     if any(name == k or name.startswith(k + ".") for k in keys)]
        live = [name for name, p in to_freeze if has_grad_slot(p)]
        if live:
            # the reference freezes inside the model constructor, before any optimizer exists; a live
            # FusedAdamW would keep writing and applying gradients of these parameters
            raise RuntimeError(f"load_pretrained_backbone(freeze=True) after FusedAdamW was built: {live[:3]}... "
                               "are in its flat groups; load (and freeze) first, then build the optimizer")
    res = backbone.load_state_dict(sd, strict=False)
    if freeze:
        for _, p in to_freeze:
            p.requires_grad = False
    invalidate_weights()
    return res.missing_keys, res.unexpected_keys


def load_model(model, src, optimizer=None):
    raw = _read(src)
    sd = raw
    for key in ("model", "state_dict", "module"):
        if isinstance(raw, dict) and key in raw:
            sd = raw[key]
            break
    if next(iter(sd), "").startswith("module."):
        sd = _strip(sd, "module.")
    model.load_state_dict(sd, strict=True)
    if optimizer is not None:
        optimizer.refresh_shadows()
    else:
        invalidate_weights()
    return model


def save_checkpoint(path, model, optimizer, epoch, iteration):
    sd = OrderedDict((k[7:] if k.split(".")[0] == "module" else k, v) for k, v in model.state_dict().items())
    torch.save({"model": sd, "optimizer": optimizer.state_dict(), "epoch": epoch, "iteration": iteration}, path)


def restore_checkpoint(path, model, optimizer):
    """Returns (next_epoch, iteration) like Engine.restore_checkpoint."""
    raw = _read(path)
    load_model(model, raw["model"], optimizer)
    optimizer.load_state_dict(raw["optimizer"])
    return raw["epoch"] + 1, raw["iteration"]
