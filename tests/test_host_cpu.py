"""Host-side logic that needs no GPU: flat-gradient slot spans, the fp16 loss-scale schedule, the
evaluate_msf input sizes and the SyncBN count cache."""
import torch
import torch.nn as nn


def test_gslot_rows_spans_adjacent_slots_only():
    from dformer_amd.functional import clear_grad_slots, gslot_rows, register_grad_slot
    clear_grad_slots()
    flat = torch.zeros(1000)
    a = nn.Parameter(torch.zeros(4, 6))
    b = nn.Parameter(torch.zeros(2, 6))
    c = nn.Parameter(torch.zeros(3, 5))
    register_grad_slot(a, flat, 0)
    register_grad_slot(b, flat, 24)       # right after a
    register_grad_slot(c, flat, 100)      # not adjacent to b
    span = gslot_rows(a, b)
    assert span is not None and span.shape == (6, 6) and span.data_ptr() == flat.data_ptr()
    span[4:].fill_(1.0)
    assert flat[24:36].eq(1.0).all() and flat[:24].eq(0.0).all()
    assert gslot_rows(b, c) is None                      # gap between the slots
    assert gslot_rows(a, c) is None
    d = nn.Parameter(torch.zeros(6))
    e = nn.Parameter(torch.zeros(2))
    register_grad_slot(d, flat, 200)
    register_grad_slot(e, flat, 206)
    v = gslot_rows(d, e)                                 # 1-D slots (biases)
    assert v is not None and v.shape == (8,)
    assert gslot_rows(a, nn.Parameter(torch.zeros(1, 6))) is None  # no slot at all
    clear_grad_slots()


def test_loss_scaler_schedule_matches_gradscaler_defaults():
    """torch.cuda.amp.GradScaler: init 2**16, x0.5 on an inf/nan step, x2 after 2000 clean steps."""
    from dformer_amd.train import LossScaler
    s = LossScaler("cpu")
    assert s.scale == 65536.0
    s.update(True)
    assert s.scale == 32768.0 and s.growth_tracker == 0 and s.skipped == 1
    for _ in range(1999):
        s.update(False)
    assert s.scale == 32768.0 and s.growth_tracker == 1999
    s.update(False)
    assert s.scale == 65536.0 and s.growth_tracker == 0


def test_msf_sizes_follow_val_mm():
    """val_mm.py:359-364: int(scale * H) rounded up to a multiple of 32."""
    from dformer_amd.evaluate import msf_size
    assert msf_size(480, 640, 1.0) == (480, 640)
    assert msf_size(480, 640, 0.75) == (384, 480)
    assert msf_size(480, 640, 1.25) == (608, 800)
    assert msf_size(530, 730, 0.5) == (288, 384)
    assert msf_size(50, 70, 0.75) == (64, 64)


def test_metrics_formulas_match_reference():
    """utils/metrics_new.py compute_iou / compute_f1 / compute_pixel_acc on a fixed histogram."""
    from dformer_amd.evaluate import Metrics
    m = Metrics(3, 255, "cpu")
    h = torch.tensor([[5, 1, 0], [2, 7, 1], [0, 0, 0]], dtype=torch.int64)
    m._hist += h.view(-1)
    ious, miou = m.compute_iou()
    hf = h.float()  # the reference keeps a float32 histogram
    want = hf.diag() / (hf.sum(0) + hf.sum(1) - hf.diag())
    want[want.isnan()] = 0
    assert ious == (want * 100).numpy().round(2).tolist() and miou == round(want.mean().item() * 100, 2)
    f1, mf1 = m.compute_f1()
    assert len(f1) == 3 and f1[2] == 0.0
    acc, macc = m.compute_pixel_acc()
    assert abs(acc[0] - 83.33) < 1e-3 and abs(macc - round((5 / 6 + 0.7) / 3 * 100, 2)) < 1e-3


def test_warmup_poly_lr():
    """WarmUpPolyLR (utils/lr_policy.py:22-34): linear warm-up to start_lr, then poly decay."""
    from dformer_amd.train import WarmUpPolyLR
    s = WarmUpPolyLR(6e-5, 0.9, 1000, 10)
    assert s.get_lr(0) == 0.0
    assert abs(s.get_lr(5) - 3e-5) < 1e-18
    assert abs(s.get_lr(10) - 6e-5 * (1 - 10 / 1000.0) ** 0.9) < 1e-18
    assert abs(s.get_lr(500) - 6e-5 * 0.5 ** 0.9) < 1e-18
    lrs = [s.get_lr(i) for i in range(10, 1000)]
    assert all(a > b for a, b in zip(lrs, lrs[1:])) and lrs[-1] > 0.0
    assert s.get_lr(1000) == 0.0


def test_frozen_chain_head_keeps_members_in_their_group():
    """A chain member (q_cut / l, proj_e, BN weight) whose chain head is frozen must still get a
    flat slot: FusedAdamW would otherwise leave it ungrouped and silently never update it."""
    import bench
    from dformer_amd.functional import clear_grad_slots
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, _chain_order, group_weight

    torch.manual_seed(0)
    model = EncoderDecoder(cfg=bench.make_cfg("DFormer-Tiny", "ham"))
    attn = model.encoder_backbone.stages[1][0].attn
    attn.q.weight.requires_grad_(False)        # head of q | q_cut | l (weights)
    attn.proj.bias.requires_grad_(False)       # head of proj | proj_e (biases)
    bn = model.decode_head.squeeze.bn
    bn.bias.requires_grad_(False)              # head of bias | weight
    decay, no_decay = group_weight(model)
    opt = FusedAdamW(model)
    try:
        grouped = {id(p) for g in opt.groups for p in g.params}
        for p in decay + no_decay:
            assert (id(p) in grouped) == p.requires_grad
        for p in (attn.q_cut.weight, attn.l.weight, attn.proj_e.bias, bn.weight):
            assert id(p) in grouped and all(p is not q for q in opt.ungrouped)
        # every parameter exactly once; untouched chains stay adjacent
        for g in opt.groups:
            assert len({id(p) for p in g.params}) == len(g.params)
        other = model.encoder_backbone.stages[1][1].attn
        g0 = opt.groups[0]
        oq, oqc, ol = (g0.slots[p][0] for p in (other.q.weight, other.q_cut.weight, other.l.weight))
        assert oqc == oq + other.q.weight.numel() and ol == oqc + other.q_cut.weight.numel()
    finally:
        clear_grad_slots()
    a, b, c, d = (torch.zeros(1, requires_grad=True) for _ in range(4))
    assert _chain_order([b, c, d], [[a, b, c]]) == [b, c, d]   # head absent: members keep their place
    assert _chain_order([c, d, a], [[a, b, c]]) == [d, a, c]   # head present, b absent: c follows a


def test_no_redefined_test_names():
    """Every test function name is defined once per test module (a redefinition silently shadows
    the first copy, so pytest would never run it)."""
    import ast
    import glob
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    for path in sorted(glob.glob(os.path.join(here, "test_*.py"))):
        with open(path) as f:
            tree = ast.parse(f.read(), path)
        names = [n.name for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef))]
        dup = sorted({n for n in names if names.count(n) > 1})
        assert not dup, f"{os.path.basename(path)} redefines {dup}"


def test_chain_order_overlapping_chains():
    """A chain member that heads a chain of its own brings that chain's tail along; chains forming
    a cycle and members whose head is absent keep every parameter exactly once."""
    from dformer_amd.train import _chain_order
    a, b, c, d, e = (nn.Parameter(torch.zeros(1)) for _ in range(5))
    order = _chain_order([a, b, c, d, e], [[a, c], [c, e]])
    assert [id(p) for p in order] == [id(a), id(c), id(e), id(b), id(d)]
    order = _chain_order([a, b, c], [[a, b], [b, a]])
    assert sorted(id(p) for p in order) == sorted(id(p) for p in (a, b, c))
    order = _chain_order([b, c, d], [[a, c, d]])  # head a not present: no regrouping
    assert [id(p) for p in order] == [id(b), id(c), id(d)]


def test_fused_ffn_env_values_are_validated():
    """DFM_FUSED_FFN maps through an explicit table; an unknown value (e.g. 'off') raises instead of
    silently selecting a fused route."""
    import pytest
    from dformer_amd.functional import _fused_ffn_mode
    assert _fused_ffn_mode("0") is False and _fused_ffn_mode("1") is True
    assert _fused_ffn_mode("fwd") == "fwd" and _fused_ffn_mode("auto") == "auto"
    for bad in ("off", "false", "true", "2", ""):
        with pytest.raises(ValueError):
            _fused_ffn_mode(bad)
