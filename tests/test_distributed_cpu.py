"""Data-parallel path on CPU: world size 2 over gloo.

The RCCL path on the GPU box uses exactly this code (train.GradBuckets / all_reduce_mean); here
the same hooks, buckets and flat gradient buffers run on CPU tensors with the gloo backend:
  * the flat gradient buffer after GradBuckets.finish() equals the SUM over ranks of each rank's
    local gradients (AdamW then scales by 1/world), for several bucket sizes (one bucket, one
    bucket per parameter, ragged);
  * every bucket is reduced exactly once per step and the per-step state resets;
  * all_reduce_mean matches pyt_utils.all_reduce_tensor (sum / world);
  * group_weight on the real DFormer-B + ham module reproduces the reference's optimizer groups.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3, padding=1)
        self.bn = nn.BatchNorm2d(8)
        self.fc1 = nn.Linear(8, 16)
        self.fc2 = nn.Linear(16, 5, bias=False)
        self.ln = nn.LayerNorm(16)
        self.extra = nn.Linear(5, 5)  # an unused branch in odd steps (its slots must be zeroed)

    def forward(self, x, use_extra=True):
        y = torch.relu(self.bn(self.conv(x))).mean(dim=(2, 3))
        out = self.fc2(self.ln(torch.relu(self.fc1(y))))
        return out + self.extra(out) if use_extra else out


def _worker(rank, world, port, bucket_bytes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dformer_amd.functional import clear_grad_slots
        from dformer_amd.train import GradBuckets, _FlatGroup, all_reduce_mean, group_weight
        torch.manual_seed(0)
        net = _Net()
        decay, no_decay = group_weight(net)
        groups = [_FlatGroup(decay, 0.01, "cpu", torch.float32), _FlatGroup(no_decay, 0.0, "cpu", torch.float32)]
        buckets = GradBuckets(groups, world, bucket_bytes)
        ok = True
        for step in range(3):
            g = torch.Generator().manual_seed(100 * rank + step)
            x = torch.randn(4, 3, 6, 7, generator=g)
            use_extra = step != 1
            # local reference gradients (a parameter copy, no hooks); no gradient = zeros
            ref = _Net()
            ref.load_state_dict(net.state_dict())
            ref(x, use_extra).square().mean().backward()
            local = {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
                     for n, p in ref.named_parameters()}
            summed = {n: t.clone() for n, t in local.items()}
            for t in summed.values():
                dist.all_reduce(t)
            # no manual zeroing of the flat buffer: finish() must clear the slots of parameters
            # whose gradient did not arrive (the `extra` branch in step 1)
            net(x, use_extra).square().mean().backward()
            buckets.finish()
            names = {id(p): n for n, p in net.named_parameters()}
            for gr in groups:
                for p, (off, k) in gr.slots.items():
                    got = gr.grad[off:off + k].view_as(p)
                    ok &= torch.allclose(got, summed[names[id(p)]], rtol=1e-5, atol=1e-6)
                    ok &= p.grad is None  # the hook handed the gradient to the flat buffer
            ok &= buckets.handles == [] and buckets.pending == [len(b[1]) for b in buckets.buckets]
            loss = torch.tensor([float(rank + 1)])
            ok &= abs(all_reduce_mean(loss, world).item() - 1.5) < 1e-6
        q.put((rank, bool(ok), len(buckets.buckets)))
        clear_grad_slots()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes", [1 << 30, 1, 700])
def test_grad_buckets_world2_gloo(bucket_bytes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, bucket_bytes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    nb = {n for _, _, n in res}
    assert len(nb) == 1
    if bucket_bytes == 1:  # one bucket per parameter
        assert nb.pop() == sum(1 for _ in _Net().parameters())


def test_group_weight_reference_groups():
    """init_func.group_weight on DFormer-B + ham: Linear/Conv weights decay; biases and BN/LN
    affine no decay; layer_scale_* and the custom LayerNorm params in no group."""
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import group_weight
    import bench
    model = EncoderDecoder(cfg=bench.make_cfg("DFormer-Base", "ham"))
    decay, no_decay = group_weight(model)
    grouped = {id(p) for p in decay + no_decay}
    left = [(n, p) for n, p in model.named_parameters() if id(p) not in grouped]
    assert all("layer_scale" in n or ".norm" in n for n, _ in left), [n for n, _ in left][:5]
    assert len(left) == 236 and sum(p.numel() for _, p in left) == 41024


def _real_model_worker(rank, world, port, q):
    """GradBuckets over the real DFormer-B + ham parameter set (CPU tensors, gloo): bucket
    membership and order, the summed gradients, and parameters that got no gradient."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from dformer_amd.functional import clear_grad_slots
        from dformer_amd.segmentor import EncoderDecoder
        from dformer_amd.train import GradBuckets, _FlatGroup, group_weight
        torch.manual_seed(0)
        model = EncoderDecoder(cfg=bench.make_cfg("DFormer-Base", "ham"))
        decay, no_decay = group_weight(model)
        groups = [_FlatGroup(decay, 0.01, "cpu", torch.float32), _FlatGroup(no_decay, 0.0, "cpu", torch.float32)]
        buckets = GradBuckets(groups, world)
        ok = []
        # membership: every grouped parameter in exactly one bucket; buckets are contiguous slices
        members = [p for _, ps in buckets.buckets for p in ps]
        ok.append(len(members) == len(set(map(id, members))) == sum(len(g.slots) for g in groups))
        for t, ps in buckets.buckets:
            g = buckets.owner[next(iter(ps))][1]
            lo = min(g.slots[p][0] for p in ps)
            hi = max(g.slots[p][0] + g.slots[p][1] for p in ps)
            ok.append(t.numel() == hi - lo == sum(g.slots[p][1] for p in ps))
            ok.append(t.numel() * 4 <= (25 << 20) + max(g.slots[p][1] for p in ps) * 4)
        # order: reverse registration within a group (the first bucket holds the last parameters)
        first = buckets.buckets[0][1]
        g0 = groups[0]
        ok.append(max(g0.slots[p][0] for p in g0.params) in {g0.slots[p][0] for p in first})
        # one backward: a per-rank random gradient for every grouped parameter except the decoder's
        # conv_seg (no gradient this step -> its slots, pre-filled with garbage, must come out zero)
        names = {id(p): n for n, p in model.named_parameters()}
        for g in groups:
            g.grad.fill_(7.0)
        skip = {id(model.decode_head.conv_seg.weight), id(model.decode_head.conv_seg.bias)}
        gen = torch.Generator().manual_seed(rank + 1)
        loss = 0.0
        want = {}
        for g in groups:
            for p in g.params:
                if id(p) in skip:
                    want[id(p)] = torch.zeros_like(p)
                    continue
                gp = torch.randn(p.shape, generator=gen)
                want[id(p)] = gp.clone()
                loss = loss + (p * gp).sum()
        for t in want.values():
            dist.all_reduce(t)
        loss.backward()
        buckets.finish()
        bad = []
        for g in groups:
            for p, (off, k) in g.slots.items():
                if not torch.allclose(g.grad[off:off + k].view_as(p), want[id(p)], rtol=1e-5, atol=1e-5):
                    bad.append(names[id(p)])
        ok.append(not bad)
        q.put((rank, all(ok), bad[:5], len(buckets.buckets)))
        clear_grad_slots()
    finally:
        dist.destroy_process_group()


def test_grad_buckets_real_model_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_real_model_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res), res
    assert len({n for *_, n in res}) == 1 and res[0][3] >= 4  # 119 MB fp32 of grads in ~25 MB buckets


def _bn_merge_model(parts, counts):
    """The algorithm of dfm_bn_merge (elementwise.hip bn_merge_kernel), restated in fp64: re-shift every
    rank's (S1, S2, K) onto rank 0's K and sum in rank order."""
    k0 = parts[0, 2].double()
    s1 = torch.zeros_like(k0)
    s2 = torch.zeros_like(k0)
    for p, n in zip(parts.double(), counts.double()):
        d = p[2] - k0
        s1 = s1 + p[0] + n * d
        s2 = s2 + p[1] + 2 * d * p[0] + n * d * d
    return torch.stack([s1, s2, k0]).float()


def test_syncbn_merge_matches_full_batch():
    """SyncBN's merge of per-shard shifted sums (the dfm_bn_merge formula) = full-batch statistics,
    for uneven shards and |mean| >> std; one shard merges to itself bit for bit."""
    torch.manual_seed(0)
    C = 24
    x = torch.randn(5000, C, dtype=torch.float64) * 0.3 + torch.linspace(-50, 80, C, dtype=torch.float64)
    cuts = [0, 700, 2900, 5000]
    parts, counts = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        xs = x[a:b]
        k = xs[0]
        d = xs - k
        parts.append(torch.stack([d.sum(0), (d * d).sum(0), k]).float())
        counts.append(b - a)
    st = _bn_merge_model(torch.stack(parts), torch.tensor(counts, dtype=torch.float32)).double()
    n = x.shape[0]
    mean = st[2] + st[0] / n
    var = st[1] / n - (st[0] / n) ** 2
    assert torch.allclose(mean, x.mean(0), rtol=1e-6, atol=1e-5)
    assert torch.allclose(var, x.var(0, unbiased=False), rtol=1e-4, atol=1e-6)
    one = _bn_merge_model(parts[0][None], torch.tensor([700.0]))
    assert torch.equal(one, parts[0])


def _unused_mismatch_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dformer_amd.functional import clear_grad_slots
        from dformer_amd.train import GradBuckets, _FlatGroup, group_weight
        torch.manual_seed(0)
        net = _Net()
        decay, no_decay = group_weight(net)
        groups = [_FlatGroup(decay, 0.01, "cpu", torch.float32), _FlatGroup(no_decay, 0.0, "cpu", torch.float32)]
        buckets = GradBuckets(groups, world, 1 << 30)
        x = torch.randn(4, 3, 6, 7)
        net(x, use_extra=(rank == 0)).square().mean().backward()  # rank 1 leaves `extra` unused
        try:
            buckets.finish()
            q.put((rank, "no error"))
        except RuntimeError as e:
            q.put((rank, "raised" if "disagree" in str(e) else str(e)))
        clear_grad_slots()
    finally:
        dist.destroy_process_group()


def test_unused_parameter_sets_must_match_across_ranks():
    """Ranks whose unused-parameter sets differ would diverge (each rank restores its own unused
    parameters while the bucket is summed): GradBuckets raises on every rank, as DDP would."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_unused_mismatch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: "raised", 1: "raised"}, res
