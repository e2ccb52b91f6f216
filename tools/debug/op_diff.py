"""Op-by-op comparison of two library builds on the fp32 e2e_tiny_small step (GPU diagnostic).

    python tools/debug/op_diff.py dump OUT.pt          records every dformer_amd.kernels call of the step (forward,
                                                       loss, backward) with host copies of its tensor outputs
    DFM_LIB_PATH=dformer_amd/variants/lib_x.so python tools/debug/op_diff.py dump OUT2.pt
    python tools/debug/op_diff.py cmp OUT.pt OUT2.pt   per call: max |a - b| / max |a| of each output, and the first
                                                       call whose outputs move by more than 1e-4 (inputs that were
                                                       bit-identical up to there point at that call)
Both builds run the same Python control flow, so call i of one run is call i of the other.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def dump(path):
    from dformer_amd import _lib, kernels as K
    from test_segmentor_gpu import fp32_audit
    print("library", _lib.LIB_PATH, "build", _lib.BUILD_TAG, flush=True)
    rec = []
    names = [n for n in dir(K) if not n.startswith("_") and callable(getattr(K, n)) and getattr(K, n).__module__ ==
             K.__name__ and n not in ("ld", "rows_of", "kernel_name", "check", "dtype_code", "ptr", "stream",
                                      "wgrad_group", "gemm_many")]
    orig = {n: getattr(K, n) for n in names}

    def wrap(n, f):
        def g(*a, **k):
            r = f(*a, **k)
            outs = r if isinstance(r, (tuple, list)) else (r,)
            # in-place outputs (out=, dx=, accumulate) are reported through the returned tensors
            torch.cuda.synchronize()
            rec.append((n, K.TAG, [t.detach().float().cpu().clone() if torch.is_tensor(t) else None for t in outs]))
            return r
        return g

    for n in names:
        setattr(K, n, wrap(n, orig[n]))
    try:
        errs = fp32_audit("e2e_tiny_small", "DFormer-Tiny", "ham", 40)
    finally:
        for n in names:
            setattr(K, n, orig[n])
    print(f"{len(rec)} calls; audit worst {max(errs.values()):.3e}")
    torch.save({"names": [r[0] for r in rec], "tags": [r[1] for r in rec], "outs": [r[2] for r in rec]}, path)


def cmp(pa, pb):
    a = torch.load(pa, weights_only=True)
    b = torch.load(pb, weights_only=True)
    assert a["names"] == b["names"], "different call sequences"
    first = None
    for i, (n, tag, oa, ob) in enumerate(zip(a["names"], a["tags"], a["outs"], b["outs"])):
        ds = []
        for x, y in zip(oa, ob):
            if x is None or y is None or x.shape != y.shape:
                continue
            ds.append(((x.double() - y.double()).abs().max() / x.double().abs().max().clamp_min(1e-30)).item())
        d = max(ds) if ds else 0.0
        if n in ("bn_apply", "linear") and oa and oa[0] is not None and oa[0].shape == ob[0].shape:
            # ReLU outputs of the two builds: elements that are zero in one and positive in the other (a
            # pre-activation within rounding of the kink) -- the backward's mask differs there
            x, y = oa[0], ob[0]
            flip = (x > 0) != (y > 0)
            if flip.any():
                v = torch.maximum(x[flip].abs(), y[flip].abs())
                print(f"      {i} {tag} {n}: {int(flip.sum())} ReLU mask flips, largest flipped value {v.max().item():.3e} "
                      f"(output max {x.abs().max().item():.3e})")
        mark = ""
        if d > 1e-4 and first is None:
            first, mark = i, "   <-- first call over 1e-4"
        if d > 1e-5 or mark or i % 50 == 0:
            print(f"{i:5d} {tag:14s} {n:24s} {d:.3e}{mark}")
    print("first call over 1e-4:", first, a["names"][first] if first is not None else None)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
