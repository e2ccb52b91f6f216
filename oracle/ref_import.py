"""Import the read-only reference (/root/reference) on CPU through oracle/ref_shims.

TEST INFRASTRUCTURE ONLY — used by oracle/make_goldens.py in the build container to
produce tests/golden/*.npz. Never imported by the product package, and never on the
GPU box (the reference does not exist there).
"""
import os
import sys

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
REF = "/root/reference"
_SHIMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_shims")


def setup():
    for p in (_SHIMS, REF):
        if p not in sys.path:
            sys.path.insert(0, p)


def import_ref():
    setup()
    import models.encoders.DFormer as dformer  # noqa: E402
    import models.decoders.ham_head as ham  # noqa: E402
    import models.decoders.MLPDecoder as mlpdec  # noqa: E402
    import models.builder as builder  # noqa: E402
    import mmcv.cnn.bricks.transformer as droppath  # noqa: E402
    return dformer, ham, mlpdec, builder, droppath
