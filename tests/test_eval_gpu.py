"""Multi-scale + flip evaluation (dformer_amd.evaluate, csrc/eval.hip) against torch / the oracle's
restatement of utils/val_mm.py:355-392 and utils/metrics_new.py:16-47."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import dformer_ref as R
import gen

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    torch.manual_seed(0)


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("src,dst", [((37, 50), (64, 96)), ((64, 96), (32, 32)), ((5, 7), (5, 7))])
def test_resize_nchw(align, flip, src, dst):
    from dformer_amd import kernels as K
    x = torch.randn(2, 6, *src, device=DEV)[:, 1:4]  # strided channel view
    y = K.resize_nchw(x, dst, align, flip=flip)
    ref = F.interpolate(x, size=dst, mode="bilinear", align_corners=align)
    if flip:
        ref = torch.flip(ref, dims=(3,))
    assert rel(y, ref) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ncls", [40, 37, 13, 64])
@pytest.mark.parametrize("flip", [False, True])
def test_msf_accumulate(dt, ncls, flip):
    from dformer_amd import kernels as K
    B, h, w, Hs, Ws, H, W = 2, 9, 12, 72, 96, 61, 83
    low = torch.randn(B, ncls, h, w, device=DEV).to(dt)
    rows = low.permute(0, 2, 3, 1).contiguous().view(-1, ncls)
    acc0 = torch.rand(B * H * W, ncls, device=DEV)
    acc = K.msf_accumulate(rows, B, h, w, ncls, (Hs, Ws), (H, W), flip, acc0.clone())
    lg = F.interpolate(low.float(), size=(Hs, Ws), mode="bilinear", align_corners=False)
    if flip:
        lg = torch.flip(lg, dims=(3,))
    lg = F.interpolate(lg, size=(H, W), mode="bilinear", align_corners=True)
    ref = acc0.view(B, H, W, ncls) + lg.softmax(1).permute(0, 2, 3, 1)
    assert rel(acc.view(B, H, W, ncls), ref) < 1e-5


def test_confusion_matches_bincount():
    from dformer_amd import kernels as K
    ncls = 40
    acc = torch.rand(3 * 50 * 70, ncls, device=DEV)
    acc[:5] = 0.5  # ties: the first maximum wins, like torch.argmax
    lab = torch.randint(0, ncls, (3, 50, 70), device=DEV)
    lab[torch.rand(3, 50, 70, device=DEV) < 0.1] = 255
    hist = torch.zeros(ncls * ncls, dtype=torch.int64, device=DEV)
    K.seg_confusion(acc, lab, ncls, 255, hist)
    K.seg_confusion(acc, lab, ncls, 255, hist)  # accumulates
    scores = acc.view(3, 50, 70, ncls).permute(0, 3, 1, 2)
    ref = R.confusion(scores.cpu(), lab.cpu(), ncls)
    assert torch.equal(hist.cpu().view(ncls, ncls), 2 * ref)


class Cfg(dict):
    __getattr__ = dict.__getitem__


@pytest.mark.parametrize("arch,dec,ncls", [("DFormer-Tiny", "ham", 40), ("DFormer-Tiny", "MLPDecoder", 37)])
def test_evaluate_msf_vs_oracle(arch, dec, ncls):
    """evaluate_msf on the HIP path (fp32, eval-mode BN with running stats, 7 NMF steps) vs the
    oracle's restatement of val_mm.py:355-392 on the same weights, bases and inputs."""
    from dformer_amd.evaluate import evaluate_msf, msf_scores
    from dformer_amd.segmentor import EncoderDecoder
    cfg = Cfg(backbone=arch, decoder=dec, decoder_embed_dim=64 if dec == "MLPDecoder" else 512, num_classes=ncls,
              drop_path_rate=0.0, bn_eps=1e-3, bn_momentum=0.1, background=255)
    model = EncoderDecoder(cfg=cfg)
    sd = model.state_dict()
    vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()])
    state = {k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in vals.items()}
    model.load_state_dict(state)
    model = model.cuda().eval()
    B, H, W = 2, 50, 70
    bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name="msf/bases")).float()
    if dec == "ham":
        model.decode_head.hamburger.ham.injected_bases = bases
    rgb_np, dep_np = gen.rgb_depth(B, H, W)
    rgb, dep = torch.from_numpy(rgb_np).float(), torch.from_numpy(dep_np).float()
    lab = torch.from_numpy(gen.labels(B, H, W, ncls))
    scales, flip = [0.75, 1.0, 1.25], True
    acc = msf_scores(model, rgb.cuda(), dep.cuda(), ncls, scales, flip)
    p = {k: v.double() for k, v in state.items() if not k.endswith("num_batches_tracked")}
    bufs = {k: v for k, v in p.items() if "running" in k}
    ref = R.msf_scores(p, arch, dec, rgb.double(), dep.double(), ncls, scales, flip, bases.double(), buffers=bufs)
    got = acc.view(B, H, W, ncls).permute(0, 3, 1, 2).cpu()
    assert rel(got, ref) < 1e-3, rel(got, ref)
    # the whole evaluate_msf loop: metrics from the HIP scores equal bincount over the same scores
    loader = [{"rgb": rgb, "modal_x": dep, "gt": lab}]
    m = evaluate_msf(model, loader, cfg, DEV, scales, flip, engine=None)
    want = R.confusion(got, lab, ncls).float()
    assert torch.equal(m.hist.cpu(), want)
    ious, miou = m.compute_iou()
    h = want.double()
    iou_ref = (h.diag() / (h.sum(0) + h.sum(1) - h.diag())).nan_to_num(0.0)
    assert abs(miou - round(iou_ref.mean().item() * 100, 2)) < 1e-6
    assert len(ious) == ncls


@pytest.mark.parametrize("name,arch,dec,ncls,embed", [("msf_tiny_ham", "DFormer-Tiny", "ham", 40, 512),
                                                      ("msf_tiny_mlp", "DFormer-Tiny", "MLPDecoder", 37, 64)])
def test_evaluate_msf_vs_reference_golden(name, arch, dec, ncls, embed):
    """The HIP evaluate_msf against the reference's own evaluate_msf (utils/val_mm.py:325-472, run by
    oracle/make_goldens.py golden_msf over two batches): the summed softmax scores of every batch at
    1e-3 (fp32) and the confusion histogram (argmax near-ties may flip a handful of pixels)."""
    from goldens import load
    from dformer_amd.evaluate import evaluate_msf, msf_scores
    from dformer_amd.segmentor import EncoderDecoder
    g = load(name)
    B, H, W, _, flip = [int(v) for v in g["meta"]]
    scales = [float(s) for s in g["scales"]]
    cfg = Cfg(backbone=arch, decoder=dec, decoder_embed_dim=embed, num_classes=ncls, drop_path_rate=0.0,
              bn_eps=1e-3, bn_momentum=0.1, background=255)
    model = EncoderDecoder(cfg=cfg)
    sd = model.state_dict()
    vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()])
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in vals.items()})
    model = model.cuda().eval()
    if dec == "ham":
        model.decode_head.hamburger.ham.injected_bases = torch.from_numpy(
            gen.nmf_bases(B, 512, 64, name=name + "/bases")).float()
    loader = []
    for i in range(2):
        rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=8964 + i)
        loader.append({"rgb": torch.from_numpy(rgb_np).float(), "modal_x": torch.from_numpy(dep_np).float(),
                       "gt": torch.from_numpy(gen.labels(B, H, W, ncls, seed=8964 + i))})
        acc = msf_scores(model, loader[-1]["rgb"].cuda(), loader[-1]["modal_x"].cuda(), ncls, scales, bool(flip))
        got = acc.view(B, H, W, ncls).permute(0, 3, 1, 2).cpu()
        assert rel(got, torch.from_numpy(g[f"scores{i}"])) < 1e-3, (i, rel(got, torch.from_numpy(g[f"scores{i}"])))
    m = evaluate_msf(model, loader, cfg, DEV, scales, bool(flip))
    ours, ref = m.hist.cpu().numpy(), g["hist"]
    valid = ref.sum()
    assert ours.sum() == valid
    assert np.abs(ours - ref).sum() / 2 <= max(2, 1e-3 * valid), np.abs(ours - ref).sum() / 2
