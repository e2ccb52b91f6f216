"""The C-ABI library loads on CPU and exports exactly what include/dformer_hip.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dformer_hip.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(?:int|size_t|const char\*)\s+(dfm_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = m.group(2).strip()
        n = 0 if args in ("", "void") else len([a for a in args.split(",") if a.strip()])
        decls[m.group(1)] = n
    return decls


def test_header_parses():
    d = declared()
    assert "dfm_gemm" in d and "dfm_pooled_attn_bwd" in d and len(d) >= 30


def test_library_exports_every_declared_symbol():
    from dformer_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared():
        assert hasattr(lib, name), name


def test_binding_signatures_match_header():
    from dformer_amd import _lib
    d = declared()
    assert set(d) == set(_lib._SIGS), set(d) ^ set(_lib._SIGS)
    for name, n in d.items():
        assert len(_lib._SIGS[name][1]) == n, (name, n, len(_lib._SIGS[name][1]))


def test_abi_version_and_error_path():
    from dformer_amd import _lib
    assert _lib.lib.dfm_abi_version() == 13
    assert _lib.BUILD_TAG.startswith("default red="), _lib.BUILD_TAG
    # argument validation fails before touching the GPU
    st = _lib.lib.dfm_layernorm_fwd(0, 10, 100000, None, 0, None, None, 1e-6, None, 0, None, None, None)
    assert st == -1
    assert b"unsupported" in _lib.lib.dfm_last_error() or b"null" in _lib.lib.dfm_last_error()
    with pytest.raises(RuntimeError):
        _lib.check(st, "dfm_layernorm_fwd")


@pytest.mark.parametrize("cname,pyname", [("DfmGemmDesc", "GemmDesc"), ("DfmPartialSum", "PartialSum"),
                                          ("DfmConvFFNDesc", "ConvFFNDesc"), ("DfmBlockDesc", "BlockDesc")])
def test_desc_layout_matches_c_struct(tmp_path, cname, pyname):
    """Each ctypes descriptor must have the C struct's size and every field offset (checked with gcc)."""
    import shutil
    import subprocess
    from dformer_amd import _lib
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    cls = getattr(_lib, pyname)
    names = [f[0] for f in cls._fields_]
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"%s\"\nint main(){printf(\"%%zu\", sizeof(%s));" % (
        HEADER, cname)
    for n in names:
        src += 'printf(" %%zu", offsetof(%s, %s));' % (cname, n)
    src += "return 0;}\n"
    (tmp_path / "t.c").write_text(src)
    subprocess.run(["gcc", str(tmp_path / "t.c"), "-o", str(tmp_path / "t")], check=True)
    vals = [int(v) for v in subprocess.run([str(tmp_path / "t")], capture_output=True, text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(cls)
    assert vals[1:] == [getattr(cls, n).offset for n in names]


def test_block_param_enum_matches_names(tmp_path):
    """BLOCK_PARAM_NAMES follows the header's DFM_BP_* enum: same count, and the enum names spell the
    reference state_dict keys in the same order."""
    import shutil
    import subprocess
    from dformer_amd import _lib
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    src = open(HEADER).read()
    start = src.index("enum {", src.index("} DfmBlockDesc;"))
    body = src[start:src.index("DFM_BLOCK_NPARAM", start)]
    enum = re.findall(r"DFM_BP_\w+", re.sub(r"/\*.*?\*/", "", body, flags=re.S))
    assert len(enum) == len(_lib.BLOCK_PARAM_NAMES)
    (tmp_path / "n.c").write_text("#include <stdio.h>\n#include \"%s\"\nint main(){printf(\"%%d\", DFM_BLOCK_NPARAM);"
                                  "return 0;}\n" % HEADER)
    subprocess.run(["gcc", str(tmp_path / "n.c"), "-o", str(tmp_path / "n")], check=True)
    assert int(subprocess.run([str(tmp_path / "n")], capture_output=True, text=True).stdout) == len(enum)
    short = {"attn.norm.weight": "NORM_W", "attn.norm_e.bias": "NORM_E_B", "attn.short_cut_linear.weight": "SC_W",
             "attn.proj_e.bias": "PROJE_B", "layer_scale_1_e": "LS1E", "mlp.pos.weight": "MLP_POS_W",
             "mlp_e2.fc2.bias": "MLPE_FC2_B"}
    for name, tag in short.items():
        assert enum[_lib.BLOCK_PARAM_NAMES.index(name)] == "DFM_BP_" + tag, name


def test_block_sizes_and_validation():
    """dfm_block_*_size plan the Block on the host (no GPU); bad descriptors are rejected before any launch."""
    from dformer_amd import _lib
    d = _lib.BlockDesc(2, 30, 40, 256, 8, 7, 1024, 0, 0, 1e-6)
    sv, ws = _lib.lib.dfm_block_saved_size(_lib.BF16, d), _lib.lib.dfm_block_workspace_size(_lib.BF16, d)
    P = 2 * 30 * 40
    assert sv > 2 * P * (256 + 1024 + 256) and ws > 0
    assert _lib.lib.dfm_block_saved_size(_lib.F32, d) > sv
    bad = _lib.BlockDesc(2, 30, 40, 250, 8, 7, 1024, 0, 0, 1e-6)
    assert _lib.lib.dfm_block_saved_size(_lib.BF16, bad) == 0
    fake = ctypes.c_void_p(1 << 20)
    st = _lib.lib.dfm_block_fwd(_lib.BF16, d, fake, None, fake, fake, fake, fake, fake, 16, fake, 16, None)
    assert st == -1 and b"needed" in _lib.lib.dfm_last_error()


@pytest.mark.parametrize("bad", [
    dict(lda=800),                      # k-contiguous A rows of K = 896 elements in an 800-element pitch
    dict(ldb=512),                      # same for B
    dict(ldc=500),                      # output rows narrower than N
    dict(stride_a=4800 * 896 - 1),      # consecutive batch matrices of A overlap
    dict(stride_b=100),
    dict(stride_c=0),                   # every batch writing one output
    dict(split_k=4, workspace_bytes=1024),  # split-K partials need 4 * 16 * 4800 * 512 * 4 bytes
    dict(out2=1 << 20, ldout2=512),     # a second output without its multiplier
    dict(out2=1 << 20, ldout2=512, mul2=1 << 20, ldmul2=512),  # ... with batch 16
])
def test_gemm_validation_rejects_bad_descriptors(bad):
    """dfm_gemm validates leading dimensions, batch strides and the workspace size before any launch
    (the NMF backward's input-gradient descriptor, ham_head.py:120-145 / decoders.py gx, perturbed)."""
    from dformer_amd import _lib
    d = dict(M=4800, N=512, K=896, batch=16, a_kcontig=1, b_kcontig=1, lda=896, ldb=896, ldc=512,
             stride_a=4800 * 896, stride_b=512 * 896, stride_c=4800 * 512, alpha=1.0, beta=0.0, rows_per_scale=1,
             workspace_bytes=0)
    d.update(bad)
    desc = _lib.GemmDesc(**d)
    fake = ctypes.c_void_p(1 << 20)  # never dereferenced: validation fails first
    st = _lib.lib.dfm_gemm(_lib.BF16, desc, fake, fake, fake, fake if "split_k" in bad else None, None)
    assert st == -1, _lib.lib.dfm_last_error()
    assert _lib.lib.dfm_last_error().startswith(b"dfm_gemm: ")
