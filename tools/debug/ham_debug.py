"""Ham-head golden debug aid (GPU only): the ham_tiny golden case, printing the error of every
input and parameter gradient (backward order) and saving the decoder's intermediates (every
autograd.Function output and the gradient flowing into it), so runs under different kernel
variants (e.g. DFM_SCALAR_RESIZE=0 vs =1) can be diffed with tools/ham_compare.py.
HAM_PERTURB=<eps> multiplies the resize+concat output by (1 + eps*N(0,1)) (sensitivity probe).

    python tools/ham_debug.py OUT.pt
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
from goldens import load, rel_err  # noqa: E402
import gen  # noqa: E402
from dformer_amd import decoders as D  # noqa: E402
from dformer_amd.functional import invalidate_weights  # noqa: E402

saved = {}
counts = {}
PERTURB = float(os.environ.get("HAM_PERTURB", "0"))


def wrap(cls, tag):
    orig = cls.apply

    def apply(*args):
        out = orig(*args)
        o = out[0] if isinstance(out, tuple) else out
        if PERTURB and tag == "ResizeCatFn":
            with torch.no_grad():
                gen_ = torch.Generator(device=o.device).manual_seed(7)
                o.mul_(1 + PERTURB * torch.randn(o.shape, device=o.device, generator=gen_))
        i = counts.get(tag, 0)
        counts[tag] = i + 1
        key = f"{tag}#{i}"
        saved[key + "/out"] = o.detach().float().cpu().clone()
        if o.requires_grad:
            o.register_hook(lambda g, key=key: saved.__setitem__(key + "/grad", g.detach().float().cpu().clone()))
        return out
    cls.apply = apply


for cname in ("ResizeCatFn", "LinearActFn", "ConvBNActFn", "NMF2DFn", "ChannelDropoutLinearFn"):
    wrap(getattr(D, cname), cname)

name = "ham_tiny"
g = load(name)
B, H, W, ncls, train, *in_ch = [int(v) for v in g["meta"]]
head = D.LightHamHead(in_channels=in_ch, num_classes=ncls, channels=512, norm_cfg=dict(type="BN"))
head.dropout_ratio = 0.0
sd = head.state_dict()
vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()])
head.load_state_dict({k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in vals.items()})
head = head.cuda().train()
invalidate_weights()
head.hamburger.ham.injected_bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name=name + "/bases")).float()
feats = [torch.from_numpy(gen.normal(name + f"/f{i}", (B, c, H >> i, W >> i))).float().cuda()
         for i, c in enumerate(in_ch)]
leaves = [f.permute(0, 2, 3, 1).contiguous().requires_grad_() for f in feats]
y = head([None] + [t.permute(0, 3, 1, 2) for t in leaves])
gy = torch.from_numpy(gen.normal(name + "/gy", tuple(y.shape))).float().cuda()
y.backward(gy)
torch.cuda.synchronize()
print("y", rel_err(y.detach().cpu(), g["y"]), flush=True)
for i, t in enumerate(leaves):
    saved[f"gf{i + 1}"] = t.grad.cpu().clone()
    print("gf", i + 1, rel_err(t.grad.permute(0, 3, 1, 2).cpu(), g[f"gf{i + 1}"]), flush=True)
for k, p in reversed(list(head.named_parameters())):
    if p.grad is None:
        continue
    a = p.grad.detach().cpu()
    saved["p/" + k] = a.clone()
    if "grad/" + k in g:
        print("grad", k, rel_err(a, g["grad/" + k]), flush=True)
    elif "gradfp/" + k in g:
        print("gradfp", k, rel_err(torch.from_numpy(gen.fingerprint(a.numpy(), 256)), g["gradfp/" + k]), flush=True)
torch.save(saved, sys.argv[1])
print("saved", len(saved), "tensors to", sys.argv[1])
