"""Diff two tools/ham_debug.py dumps (e.g. DFM_SCALAR_RESIZE=0 vs =1): relative L2 difference of
every saved tensor in recording order, and the number of elements whose zero / non-zero pattern
differs (a ReLU kink taken on the other side).

    python tools/ham_compare.py gpurun_out/hd0.pt gpurun_out/hd1.pt
"""
import sys

import torch


def main():
    a = torch.load(sys.argv[1], weights_only=True)
    b = torch.load(sys.argv[2], weights_only=True)
    for k, va in a.items():
        vb = b.get(k)
        if vb is None or vb.shape != va.shape:
            continue
        da, db = va.double(), vb.double()
        rel = float((da - db).norm() / db.norm().clamp_min(1e-30))
        flips = int(((da == 0) != (db == 0)).sum())
        print(f"{k:44s} {str(tuple(va.shape)):22s} rel {rel:.3e}  zero-pattern diffs {flips}")


if __name__ == "__main__":
    main()
