"""Generate tests/golden/*.npz by running the READ-ONLY reference on CPU in float64.

TEST INFRASTRUCTURE. Run in the build container only:
    PYTHONDONTWRITEBYTECODE=1 python oracle/make_goldens.py
It imports /root/reference through oracle/ref_shims (mmcv/mmengine restatements),
loads deterministic weights from oracle/gen.py, and stores forward outputs and
upstream-grad-seeded backward results. Nothing from the reference is copied: the
.npz files hold only arrays (inputs are regenerated from the seeds in gen.py).

Routing around HEAD's crashes: the backbone's `(outs, None)` tuple is
indexed with [0] before the decode head, and the loss of builder.py:230 is applied
by hand.
"""
import contextlib
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen  # noqa: E402
import ref_import  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
torch.set_default_dtype(torch.float64)
dformer, ham, mlpdec, builder, droppath = ref_import.import_ref()

BN = dict(type="BN", requires_grad=True)
MODELS = {  # DFormer.py:460-497
    "tiny": dict(dims=[32, 64, 128, 256], heads=[1, 2, 4, 8], ratios=[8, 8, 4, 4], depths=[3, 3, 5, 2]),
    "base": dict(dims=[64, 128, 256, 512], heads=[1, 2, 4, 8], ratios=[8, 8, 4, 4], depths=[3, 3, 12, 2]),
    "large": dict(dims=[96, 192, 288, 576], heads=[1, 2, 4, 8], ratios=[8, 8, 4, 4], depths=[3, 3, 12, 2]),
}


def load_weights(mod, seed=1234):
    sd = mod.state_dict()
    vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()], seed)
    mod.load_state_dict({k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in vals.items()})


def t(a, grad=True):
    x = torch.from_numpy(np.asarray(a, dtype=np.float64)).clone()
    return x.requires_grad_(grad)


def param_grads(mod, prefix="grad/", big=65536):
    """Full grads for small tensors; 256-sample fingerprints ("gradfp/") for large ones."""
    out = {}
    for n, p in mod.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().numpy()
        if g.size > big:
            out["gradfp/" + n] = gen.fingerprint(g, 256)
        else:
            out[prefix + n] = g.astype(np.float32)
    return out


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"  wrote {name}.npz ({os.path.getsize(path) / 1e6:.2f} MB)")


def make_block(model, stage, last=False, drop_prob=0.0):
    m = MODELS[model]
    C = m["dims"][stage]
    depth = m["depths"][stage]
    j = depth - 1 if last else 0
    return dformer.Block(index=0, dim=C, num_head=m["heads"][stage], norm_cfg=BN,
                         mlp_ratio=m["ratios"][stage], block_index=depth - j, last_block_index=50,
                         window=0 if stage == 0 else 7,
                         dropout_layer=dict(type="DropPath", drop_prob=drop_prob),
                         drop_depth=(stage == 3 and last))


def golden_block(name, model, stage, B, H, W, last=False, drop_prob=0.0, masks=None, with_ye=False):
    """One Block's output, input gradients and parameter gradients (fp64) under a seeded linear loss.
    with_ye (a drop_depth Block): x_e's output (the attention's e_back result, DFormer.py:133, 141-145,
    177-181) is in the loss and stored too, although the encoder discards it after the last Block."""
    C = MODELS[model]["dims"][stage]
    blk = make_block(model, stage, last, drop_prob)
    load_weights(blk)
    blk.train()
    x = t(gen.normal(name + "/x", (B, H, W, C)))
    xe = t(gen.normal(name + "/xe", (B, H, W, C // 2)))
    if masks is not None:
        droppath.INJECTED_MASKS = [torch.tensor(mk, dtype=torch.float64) for mk in masks]
    y, ye = blk(x, xe)
    droppath.INJECTED_MASKS = None
    gy = gen.normal(name + "/gy", y.shape)
    loss = (y * t(gy, False)).sum()
    extra = {}
    if not last or with_ye:
        gye = gen.normal(name + "/gye", ye.shape)
        loss = loss + (ye * t(gye, False)).sum()
        extra["y_e"] = ye.detach().numpy().astype(np.float32)
    loss.backward()
    save(name, y=y.detach().numpy().astype(np.float32), gx=x.grad.numpy().astype(np.float32),
         gxe=x.grad.new_zeros(0).numpy() if xe.grad is None else xe.grad.numpy().astype(np.float32),
         meta=np.array([B, H, W, C, stage, int(last), drop_prob * 1e6]), **extra, **param_grads(blk))


def golden_block_bf16_env(name, model, stage, B, H, W, last=False):
    """The reference Block's OWN bf16 error (float32 weights / inputs under torch.autocast(bfloat16)
    on CPU) against the fp64 golden `name`, per output: y, y_e, gx, gxe and every parameter gradient,
    with the statistics the GPU gates use (rel-to-max for full tensors, tests/goldens.py fp_rel_err
    for fingerprinted ones). tests/test_block_gpu.py gates the HIP bf16 Block at a stated multiple
    of this envelope (a bf16 gate must be per Block and relative to what bf16 can do)."""
    g = dict(np.load(os.path.join(OUT, name + ".npz")))
    C = MODELS[model]["dims"][stage]
    blk = make_block(model, stage, last)
    load_weights(blk)
    blk = blk.float().train()
    x = torch.from_numpy(gen.normal(name + "/x", (B, H, W, C))).float().requires_grad_()
    xe = torch.from_numpy(gen.normal(name + "/xe", (B, H, W, C // 2))).float().requires_grad_()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        y, ye = blk(x, xe)
    loss = (y.float() * torch.from_numpy(gen.normal(name + "/gy", y.shape)).float()).sum()
    if not last:
        loss = loss + (ye.float() * torch.from_numpy(gen.normal(name + "/gye", ye.shape)).float()).sum()
    loss.backward()

    def rel(a, b):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)

    env = {"env/y": rel(y.detach().double().numpy(), g["y"]), "env/gx": rel(x.grad.double().numpy(), g["gx"])}
    if not last:
        env["env/y_e"] = rel(ye.detach().double().numpy(), g["y_e"])
        env["env/gxe"] = rel(xe.grad.double().numpy(), g["gxe"])
    for n, p in blk.named_parameters():
        if p.grad is None:
            continue
        a = p.grad.detach().double().numpy()
        if "grad/" + n in g:
            b = g["grad/" + n].astype(np.float64)
            if np.abs(b).max() < 1e-12:  # mathematically zero gradient (fp64 noise): not gated
                continue
            env["env/grad/" + n] = rel(a, b)
        elif "gradfp/" + n in g:
            env["env/grad/" + n] = _fp_rel_err(gen.fingerprint(a, 256), g["gradfp/" + n])
    gv = np.array([v for k, v in env.items() if k.startswith("env/grad/")])
    print(f"  bf16env {name}: y {env['env/y']:.3e} gx {env['env/gx']:.3e} param-grad median {np.median(gv):.3e} "
          f"max {gv.max():.3e}")
    save("bf16env_" + name, **{k: np.array(v) for k, v in env.items()})


def golden_nmf(name, B, C, H, W, train=True):
    nmf = ham.NMF2D(dict(device="cpu"))
    nmf.train(train)
    bases = gen.nmf_bases(B, C, 64, name=name + "/bases")
    nmf._build_bases = lambda B_, S, D, R, cuda=False: torch.from_numpy(bases.copy())
    x = t(gen.uniform(name + "/x", (B, C, H, W)))
    y = nmf(x)
    gy = gen.normal(name + "/gy", y.shape)
    (y * t(gy, False)).sum().backward()
    save(name, y=y.detach().numpy().astype(np.float32), gx=x.grad.numpy().astype(np.float32),
         meta=np.array([B, C, H, W, int(train)]))


def _ham_head(in_ch, ncls, train):
    head = ham.LightHamHead(in_channels=in_ch, num_classes=ncls, in_index=[1, 2, 3], norm_cfg=BN,
                            channels=512, device="cpu")
    for mdl in head.modules():  # init_func.py:11-15 applies bn_eps / momentum to the decoder
        if isinstance(mdl, nn.BatchNorm2d):
            mdl.eps, mdl.momentum = 1e-3, 0.1
    head.dropout = None  # value golden: Dropout2d removed (p=0)
    load_weights(head)
    head.train(train)
    return head


def _relu_margins(head, tag, in_ch, B, H, W):
    """min |input| / max |input| over each of the head's four ReLUs (squeeze, ham_in, the
    Hamburger's relu(x + ham_out), align) for the inputs drawn under `tag`."""
    seen = {}
    hooks = [head.squeeze.activate.register_forward_pre_hook(lambda m, a: seen.__setitem__("squeeze", a[0].clone())),
             head.align.activate.register_forward_pre_hook(lambda m, a: seen.__setitem__("align", a[0].clone())),
             head.hamburger.ham_in.register_forward_hook(lambda m, a, o: seen.__setitem__("ham_in", o.clone())),
             head.hamburger.register_forward_pre_hook(lambda m, a: seen.__setitem__("x", a[0].clone())),
             head.hamburger.ham_out.register_forward_hook(lambda m, a, o: seen.__setitem__("ham_out", o.clone()))]
    bases = gen.nmf_bases(B, 512, 64, name=tag + "/bases")
    head.hamburger.ham._build_bases = lambda B_, S, D, R, cuda=False: torch.from_numpy(bases.copy())
    with torch.no_grad():
        head([None] + [t(gen.normal(tag + f"/f{i}", (B, c, H >> i, W >> i)), False) for i, c in enumerate(in_ch)])
    for h in hooks:
        h.remove()
    seen["ham"] = seen.pop("x") + seen.pop("ham_out")
    return min((v.abs().min() / v.abs().max()).item() for v in seen.values())


def golden_ham(name, in_ch, B, H, W, ncls=40, train=True, margin=1e-5, tries=400):
    """LightHamHead golden whose inputs keep every ReLU input at least `margin` x max away from
    the kink: the HIP fp32 path then sees the same activation pattern as fp64 and every gradient
    behind the Hamburger's ReLU is gated at 1e-3 (round 1's fixture sat on the kink)."""
    head = _ham_head(in_ch, ncls, train)
    for s in range(tries):
        tag = f"{name}#{s}"
        mg = _relu_margins(head, tag, in_ch, B, H, W)
        if mg > margin:
            break
    else:
        raise RuntimeError(f"no input seed with ReLU margin > {margin}")
    print(f"  {name}: input seed {s}, ReLU margin {mg:.2e}")
    head = _ham_head(in_ch, ncls, train)
    bases = gen.nmf_bases(B, 512, 64, name=tag + "/bases")
    head.hamburger.ham._build_bases = lambda B_, S, D, R, cuda=False: torch.from_numpy(bases.copy())
    feats = [t(gen.normal(tag + f"/f{i}", (B, c, H >> i, W >> i))) for i, c in enumerate(in_ch)]
    inputs = [None] + feats
    y = head(inputs)
    gy = gen.normal(tag + "/gy", y.shape)
    (y * t(gy, False)).sum().backward()
    extra = {}
    for n, b in head.named_buffers():
        if "running" in n:
            extra["buf/" + n] = b.numpy().astype(np.float32)
    save(name, y=y.detach().numpy().astype(np.float32),
         **{f"gf{i + 1}": f.grad.numpy().astype(np.float32) for i, f in enumerate(feats)},
         meta=np.array([B, H, W, ncls, int(train), s] + list(in_ch)), margin=np.array(mg),
         **param_grads(head), **extra)


def golden_mlpdec(name, in_ch, B, H, W, embed, ncls=40):
    head = mlpdec.DecoderHead(in_channels=in_ch, num_classes=ncls, norm_layer=nn.BatchNorm2d,
                              embed_dim=embed)
    for mdl in head.modules():
        if isinstance(mdl, nn.BatchNorm2d):
            mdl.eps, mdl.momentum = 1e-3, 0.1
    head.dropout = nn.Identity()
    load_weights(head)
    head.train()
    sizes = [(H, W)]
    for _ in range(3):
        h, w = sizes[-1]
        sizes.append(((h - 1) // 2 + 1, (w - 1) // 2 + 1))
    feats = [t(gen.normal(name + f"/f{i}", (B, c, *sizes[i]))) for i, c in enumerate(in_ch)]
    y = head(feats)
    gy = gen.normal(name + "/gy", y.shape)
    (y * t(gy, False)).sum().backward()
    save(name, y=y.detach().numpy().astype(np.float32),
         **{f"gf{i}": f.grad.numpy().astype(np.float32) for i, f in enumerate(feats)},
         meta=np.array([B, H, W, ncls, embed] + list(in_ch)), **param_grads(head))


class Cfg(dict):
    __getattr__ = dict.__getitem__


def build_segmentor(backbone, decoder="ham", ncls=40, embed=512):
    cfg = Cfg(backbone=backbone, decoder=decoder, decoder_embed_dim=embed, num_classes=ncls,
              drop_path_rate=0.0, aux_rate=0, device="cpu", pretrained_model=None, bn_eps=1e-3,
              bn_momentum=0.1, background=255)
    crit = nn.CrossEntropyLoss(reduction="none", ignore_index=255)
    model = builder.EncoderDecoder(cfg=cfg, criterion=crit, norm_layer=nn.BatchNorm2d, syncbn=False)
    if decoder == "ham":
        model.decode_head.dropout = None
    else:
        model.decode_head.dropout = nn.Identity()
    load_weights(model)
    return model, cfg


def e2e_forward(model, rgb, dep, bases=None):
    """encode_decode of builder.py:193-208 with the HEAD tuple bug routed around."""
    if bases is not None:
        model.decode_head.hamburger.ham._build_bases = \
            lambda B_, S, D, R, cuda=False: torch.from_numpy(bases.copy())
    feats = model.encoder_backbone(rgb, dep)[0]
    low = model.decode_head.forward(feats)
    out = F.interpolate(low, size=rgb.shape[-2:], mode="bilinear", align_corners=False)
    return feats, low, out


def _e2e_relu_margin(model, B, H, W, seed, bases):
    """min |input| / max |input| over the ham head's four ReLUs (as _relu_margins) for the inputs drawn
    with `seed`, in the training-mode forward."""
    head = model.decode_head
    seen = {}
    hooks = [head.squeeze.activate.register_forward_pre_hook(lambda m, a: seen.__setitem__("squeeze", a[0].clone())),
             head.align.activate.register_forward_pre_hook(lambda m, a: seen.__setitem__("align", a[0].clone())),
             head.hamburger.ham_in.register_forward_hook(lambda m, a, o: seen.__setitem__("ham_in", o.clone())),
             head.hamburger.register_forward_pre_hook(lambda m, a: seen.__setitem__("x", a[0].clone())),
             head.hamburger.ham_out.register_forward_hook(lambda m, a, o: seen.__setitem__("ham_out", o.clone()))]
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=seed)
    sd = {k: v.clone() for k, v in model.state_dict().items()}  # the running statistics move in train mode
    with torch.no_grad():
        e2e_forward(model, t(rgb_np, False), t(dep_np, False), bases)
    model.load_state_dict(sd)
    for h in hooks:
        h.remove()
    seen["ham"] = seen.pop("x") + seen.pop("ham_out")
    return min((v.abs().min() / v.abs().max()).item() for v in seen.values())


def golden_e2e(name, backbone, B, H, W, decoder="ham", ncls=40, embed=512, backward=True, margin=None, tries=200):
    """End-to-end golden (features, logits, loss, input and parameter gradient fingerprints). With `margin`
    (ham decoder) the input draw is the first seed from 8964 whose decoder ReLU inputs all stay at least
    margin x max away from the kink, so an fp32 run cannot flip an activation against fp64 by summation
    order alone (round 5's e2e_tiny_small had one align-ReLU input at 6e-7 of max: a reduction-geometry
    change flipped it and moved every gradient behind it by up to 1.2e-2); the seed is meta[4]."""
    t0 = time.time()
    model, cfg = build_segmentor(backbone, decoder, ncls, embed)
    model.train()
    seed = 8964
    if margin is not None:
        bases0 = gen.nmf_bases(B, 512, 64, name=name + "/bases")
        for seed in range(8964, 8964 + tries):
            mg = _e2e_relu_margin(model, B, H, W, seed, bases0)
            if mg > margin:
                break
        else:
            raise RuntimeError(f"no input seed with ReLU margin > {margin}")
        print(f"  {name}: input seed {seed}, decoder ReLU margin {mg:.2e}")
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=seed)
    rgb, dep = t(rgb_np, backward), t(dep_np, backward)
    lab = torch.from_numpy(gen.labels(B, H, W, ncls))
    bases = gen.nmf_bases(B, 512, 64, name=name + "/bases") if decoder == "ham" else None
    if not backward:
        with torch.no_grad():
            feats, low, out = e2e_forward(model, rgb, dep, bases)
        save(name, low_fp=gen.fingerprint(low.numpy()), out_fp=gen.fingerprint(out.numpy()),
             **{f"feat{i}_fp": gen.fingerprint(f.numpy()) for i, f in enumerate(feats)},
             meta=np.array([B, H, W, ncls]))
        print(f"  {name}: {time.time() - t0:.1f}s")
        return
    feats, low, out = e2e_forward(model, rgb, dep, bases)
    loss = model.criterion(out, lab.long())[lab.long() != cfg.background].mean()  # builder.py:230
    loss.backward()
    gfp = {"gfp/" + n: gen.fingerprint(p.grad.numpy(), 16) for n, p in model.named_parameters()
           if p.grad is not None}
    save(name, low=low.detach().numpy().astype(np.float32), loss=np.array(loss.item()),
         grgb_fp=gen.fingerprint(rgb.grad.numpy()), gdep_fp=gen.fingerprint(dep.grad.numpy()),
         **{f"feat{i}": f.detach().numpy().astype(np.float32) for i, f in enumerate(feats)},
         meta=np.array([B, H, W, ncls] + ([seed] if margin is not None else [])), **gfp)
    print(f"  {name}: {time.time() - t0:.1f}s")


def _fp_rel_err(fa, fb, atol=1e-9):
    """Same statistic as tests/goldens.py fp_rel_err (sum / abs-sum / l2 / relative L2 of the samples)."""
    fa, fb = np.asarray(fa, np.float64), np.asarray(fb, np.float64)
    return max(abs(fa[0] - fb[0]) / max(fb[1], atol), abs(fa[1] - fb[1]) / max(fb[1], atol),
               abs(fa[2] - fb[2]) / max(fb[2], atol),
               np.linalg.norm(fa[3:] - fb[3:]) / max(np.linalg.norm(fb[3:]), atol))


def golden_bf16_env(name, backbone, B, H, W, decoder="ham", ncls=40, embed=512, dtype=torch.bfloat16,
                    prefix="bf16env_"):
    """The reference's OWN bf16 error on an e2e golden: the same model, weights and inputs run in
    float32 under torch.autocast(bfloat16) on CPU (what train.py's --amp does with bf16), compared
    with the fp64 golden. The HIP bf16 path is gated against this envelope (reference
    bf16 autocast misses a plain 1e-2 end-to-end gate by itself)."""
    g = dict(np.load(os.path.join(OUT, name + ".npz")))
    model, cfg = build_segmentor(backbone, decoder, ncls, embed)
    model = model.float().train()
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=int(g["meta"][4]) if g["meta"].size > 4 else 8964)
    rgb = torch.from_numpy(rgb_np).float().requires_grad_()
    dep = torch.from_numpy(dep_np).float().requires_grad_()
    lab = torch.from_numpy(gen.labels(B, H, W, ncls)).long()
    bases = gen.nmf_bases(B, 512, 64, name=name + "/bases") if decoder == "ham" else None
    if bases is not None:
        model.decode_head.hamburger.ham._build_bases = \
            lambda B_, S, D, R, cuda=False: torch.from_numpy(bases.astype(np.float32))
    with (torch.autocast("cpu", dtype=dtype) if dtype is not None else contextlib.nullcontext()):
        feats = model.encoder_backbone(rgb, dep)[0]
        low = model.decode_head.forward(feats)
        out = F.interpolate(low, size=rgb.shape[-2:], mode="bilinear", align_corners=False)
    loss = model.criterion(out.float(), lab)[lab != cfg.background].mean()
    loss.backward()
    lowg = g["low"].astype(np.float64)
    env = {"env/low": np.abs(low.detach().double().numpy() - lowg).max() / np.abs(lowg).max(),
           "env/loss": abs(loss.item() - float(g["loss"])) / abs(float(g["loss"])),
           "env/grgb": _fp_rel_err(gen.fingerprint(rgb.grad.double().numpy()), g["grgb_fp"])}
    for n, p in model.named_parameters():
        if p.grad is not None and "gfp/" + n in g:
            env["env/gfp/" + n] = _fp_rel_err(gen.fingerprint(p.grad.double().numpy(), 16), g["gfp/" + n], atol=1e-4)
    gv = np.array([v for k, v in env.items() if k.startswith("env/gfp/")])
    print(f"  {prefix} envelope {name}: low {env['env/low']:.3e} loss {env['env/loss']:.3e} grgb {env['env/grgb']:.3e} "
          f"param-grad median {np.median(gv):.3e} p90 {np.quantile(gv, 0.9):.3e} max {gv.max():.3e}")
    save(prefix + name, **{k: np.array(v) for k, v in env.items()})


def golden_msf(name, backbone, B, H, W, decoder="ham", ncls=40, embed=512, scales=(0.75, 1.0, 1.25), flip=True):
    """The reference's own evaluate_msf (utils/val_mm.py:325-472) over two batches with the model in
    eval mode (encode_decode with the HEAD tuple bug routed around; NMF bases injected): the summed
    softmax scores handed to Metrics.update and the final confusion histogram."""
    import utils.val_mm as val_mm  # noqa: E402  (the reference, read-only)
    t0 = time.time()
    model, cfg = build_segmentor(backbone, decoder, ncls, embed)
    model.eval()
    bases = gen.nmf_bases(B, 512, 64, name=name + "/bases") if decoder == "ham" else None

    class Wrapped(nn.Module):
        def __init__(self):
            super().__init__()
            self.m = model

        def forward(self, rgb, dep):
            return e2e_forward(self.m, rgb, dep, bases)[2]

    captured = []

    class RecMetrics(val_mm.Metrics):
        def update(self, pred, target):
            captured.append(pred.detach().clone())
            super().update(pred, target)

    val_mm.Metrics = RecMetrics
    loader = []
    for i in range(2):
        rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=8964 + i)
        loader.append({"rgb": torch.from_numpy(rgb_np), "modal_x": torch.from_numpy(dep_np),
                       "gt": torch.from_numpy(gen.labels(B, H, W, ncls, seed=8964 + i)).long(), "fn": ["x.png"]})
    config = Cfg(num_classes=ncls, background=255, dataset_name="NYUDepthv2")
    engine = Cfg(distributed=False, local_rank=0)
    with torch.no_grad():
        metrics = val_mm.evaluate_msf(Wrapped(), loader, config, torch.device("cpu"), list(scales), flip, engine)
    save(name, scores0=captured[0].numpy().astype(np.float32), scores1=captured[1].numpy().astype(np.float32),
         hist=metrics.hist.numpy(), scales=np.array(scales), meta=np.array([B, H, W, ncls, int(flip)]))
    print(f"  {name}: {time.time() - t0:.1f}s")


def golden_groups():
    """Optimizer-group membership of group_weight (init_func.py:26-70) for Base + ham."""
    from utils.init_func import group_weight
    model, _ = build_segmentor("DFormer-Base")
    groups = group_weight([], model, nn.BatchNorm2d, 6e-5)
    ids = {id(p): n for n, p in model.named_parameters()}
    decay = sorted(ids[id(p)] for p in groups[0]["params"])
    nodecay = sorted(ids[id(p)] for p in groups[1]["params"])
    excluded = sorted(set(ids.values()) - set(decay) - set(nodecay))
    save("groups_base", decay=np.array(decay), nodecay=np.array(nodecay), excluded=np.array(excluded),
         counts=np.array([sum(p.numel() for n, p in model.named_parameters() if n in excluded),
                          sum(p.numel() for p in model.parameters())]))


def main():
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:]

    def want(n):
        return not which or any(n.startswith(w) for w in which)

    torch.manual_seed(0)
    blocks = [
        ("block_tiny_s0", "tiny", 0, 2, 12, 16, False),
        ("block_tiny_s1", "tiny", 1, 2, 11, 13, False),
        ("block_tiny_s3_last", "tiny", 3, 2, 5, 7, True),
        ("block_base_s0", "base", 0, 1, 16, 20, False),
        # the stage-0 plane of a 480x640 image (19,200 pixels): the fused ConvFFN's "auto" mode runs here
        ("block_base_s0_120x160", "base", 0, 1, 120, 160, False),
        ("block_base_s1", "base", 1, 2, 15, 20, False),
        ("block_base_s2", "base", 2, 2, 9, 10, False),
        ("block_base_s3", "base", 3, 2, 8, 10, False),
        ("block_base_s3_last", "base", 3, 2, 8, 10, True),
        ("block_large_s1", "large", 1, 1, 9, 11, False),
        ("block_large_s2", "large", 2, 1, 8, 9, False),
        # DFormer-Large at 530x730 (BASELINE config 5): stage 2 is 34x46, stage 3 17x23
        ("block_large_s2_34x46", "large", 2, 1, 34, 46, False),
        ("block_large_s3_17x23", "large", 3, 1, 17, 23, False),
    ]
    for n, mdl, st, B, H, W, last in blocks:
        if want(n):
            golden_block(n, mdl, st, B, H, W, last)
    if want("block_tiny_s3_last_ye"):
        golden_block("block_tiny_s3_last_ye", "tiny", 3, 2, 5, 7, True, with_ye=True)
    if want("block_droppath"):
        # DropPath with injected keep masks: 6 DropPath calls per block (x/xe × attn/mlp … order of Block.forward)
        masks = [np.array([1.0, 0.0]), np.array([0.0, 1.0]), np.array([1.0, 1.0]), np.array([0.0, 1.0])]
        golden_block("block_droppath_base_s1", "base", 1, 2, 9, 11, False, drop_prob=0.25, masks=masks)
    if want("nmf"):
        golden_nmf("nmf_train", 2, 64, 8, 10, True)
        golden_nmf("nmf_eval", 1, 64, 7, 9, False)
    if want("ham"):
        golden_ham("ham_tiny", [64, 128, 256], 1, 6, 8)
    if want("mlpdec"):
        golden_mlpdec("mlpdec_small", [32, 64, 128, 256], 2, 16, 20, embed=64)
    if want("e2e_tiny_small"):
        golden_e2e("e2e_tiny_small", "DFormer-Tiny", 2, 64, 96, margin=3e-6)
    if want("e2e_base_small"):
        golden_e2e("e2e_base_small", "DFormer-Base", 2, 64, 80)
    if want("e2e_large_mlp"):
        golden_e2e("e2e_large_mlp_small", "DFormer-Large", 1, 53, 73, decoder="MLPDecoder", ncls=37)
    if want("e2e_tiny_full"):
        golden_e2e("e2e_tiny_full_fwd", "DFormer-Tiny", 2, 480, 640, backward=False)
    if want("groups"):
        golden_groups()
    if want("msf"):
        golden_msf("msf_tiny_ham", "DFormer-Tiny", 2, 50, 70)
        golden_msf("msf_tiny_mlp", "DFormer-Tiny", 1, 45, 61, decoder="MLPDecoder", ncls=37, embed=64)
    if want("bf16env_block"):
        for n, mdl, st, B, H, W, last in blocks:
            if n in ("block_tiny_s1", "block_base_s0", "block_base_s1", "block_base_s2", "block_base_s3",
                     "block_base_s3_last", "block_large_s2", "block_base_s0_120x160"):
                golden_block_bf16_env(n, mdl, st, B, H, W, last)
    if want("bf16env") and not which == ["bf16env_block"]:
        golden_bf16_env("e2e_tiny_small", "DFormer-Tiny", 2, 64, 96)
        golden_bf16_env("e2e_base_small", "DFormer-Base", 2, 64, 80)
        golden_bf16_env("e2e_large_mlp_small", "DFormer-Large", 1, 53, 73, decoder="MLPDecoder", ncls=37)
    if want("fp32env"):  # the reference's own float32 error vs fp64: the noise floor of the fp32 gates
        golden_bf16_env("e2e_tiny_small", "DFormer-Tiny", 2, 64, 96, dtype=None, prefix="fp32env_")
        golden_bf16_env("e2e_base_small", "DFormer-Base", 2, 64, 80, dtype=None, prefix="fp32env_")
        golden_bf16_env("e2e_large_mlp_small", "DFormer-Large", 1, 53, 73, decoder="MLPDecoder", ncls=37,
                        dtype=None, prefix="fp32env_")
    if want("f16env"):  # the reference's own torch.autocast(float16) error (train.py --amp, config 5)
        golden_bf16_env("e2e_large_mlp_small", "DFormer-Large", 1, 53, 73, decoder="MLPDecoder", ncls=37,
                        dtype=torch.float16, prefix="f16env_")


if __name__ == "__main__":
    main()
