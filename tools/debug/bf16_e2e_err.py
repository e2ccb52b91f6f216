"""Diagnostic: bf16 end-to-end logits / loss error vs the fp64 golden for one e2e golden
(argv: name arch dec ncls). Run with DFM_FUSED_FFN=0/1 to A/B the fused ConvFFN."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import gen  # noqa: E402
from goldens import load, rel_err  # noqa: E402
from test_segmentor_gpu import build  # noqa: E402

name, arch, dec, ncls = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
g = load(name)
B, H, W, _ = [int(v) for v in g["meta"]]
model = build(arch, dec, ncls, "cuda").set_compute_dtype(torch.bfloat16).train()
if dec == "ham":
    model.decode_head.hamburger.ham.injected_bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name=name + "/bases")).float()
rgb_np, dep_np = gen.rgb_depth(B, H, W)
rgb = torch.from_numpy(rgb_np).float().cuda()
dep = torch.from_numpy(dep_np).float().cuda()
with torch.no_grad():
    feats = model.encoder_backbone(rgb, dep)[0]
    low = model.decode_head(feats)
print(os.environ.get("DFM_FUSED_FFN", "1"), name, "low", rel_err(low.float().cpu(), g["low"]),
      *[("feat%d" % i, round(rel_err(f.float().cpu(), g[f"feat{i}"]), 5)) for i, f in enumerate(feats)])
