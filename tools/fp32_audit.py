"""Where does the fp32 HIP path lose precision? (diagnostic, GPU)

Runs a golden case (default e2e_tiny_small: DFormer-Tiny + ham, 2x64x96) forward + loss + backward
on the HIP path in float32 and the oracle restatement in float64 on the host, and prints the
relative-to-max error of every intermediate the two share (tests/test_segmentor_gpu.py fp32_audit):
encoder features and their gradients, the low-res logits and their gradient, the image gradients
and the worst parameter gradients. The reference's own fp32 error on the same case is ~1e-6
(tests/golden/fp32env_e2e_tiny_small.npz).

    python tools/fp32_audit.py [name arch decoder ncls]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from test_segmentor_gpu import fp32_audit  # noqa: E402


def main():
    name, arch, dec, ncls = (sys.argv[1:5] if len(sys.argv) > 4 else ("e2e_tiny_small", "DFormer-Tiny", "ham", "40"))
    errs = fp32_audit(name, arch, dec, int(ncls))
    for k in sorted(k for k in errs if not k.startswith("grad/")):
        print(f"{errs[k]:.3e}  {k}")
    pg = sorted(((v, k) for k, v in errs.items() if k.startswith("grad/")), reverse=True)
    print(f"parameter gradients: {len(pg)}; worst:")
    for v, k in pg[:15]:
        print(f"   {v:.3e}  {k[5:]}")


if __name__ == "__main__":
    main()
