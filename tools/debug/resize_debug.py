"""A/B check of the resize+concat path of the ham head (vector vs DFM_SCALAR_RESIZE kernels)."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dformer_amd import kernels as K
from dformer_amd.decoders import ResizeCatFn
torch.manual_seed(0)
B = 2
chans, hws = [64, 128, 256], [(12, 16), (6, 8), (3, 4)]
feats = [torch.randn(B * h * w, c, device="cuda") for c, (h, w) in zip(chans, hws)]
for f in feats:
    f.requires_grad_()
out = ResizeCatFn.apply(B, hws, *feats)
g = torch.randn_like(out)
out.backward(g)
torch.save({"out": out.detach().cpu(), "g": [f.grad.cpu() for f in feats]}, sys.argv[1])
print("saved", sys.argv[1], float(out.abs().sum()), [float(f.grad.abs().sum()) for f in feats])
