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

    def forward(self, x):
        y = torch.relu(self.bn(self.conv(x))).mean(dim=(2, 3))
        return self.fc2(self.ln(torch.relu(self.fc1(y))))


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
        for step in range(2):
            g = torch.Generator().manual_seed(100 * rank + step)
            x = torch.randn(4, 3, 6, 7, generator=g)
            # local reference gradients (a parameter copy, no hooks)
            ref = _Net()
            ref.load_state_dict(net.state_dict())
            ref(x).square().mean().backward()
            local = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
            summed = {n: t.clone() for n, t in local.items()}
            for t in summed.values():
                dist.all_reduce(t)
            for gr in groups:
                gr.grad.zero_()
            net(x).square().mean().backward()
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
