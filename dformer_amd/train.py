"""One data-parallel training step of utils/train.py:309-383 on HIP kernels + RCCL.

  group_weight      utils/init_func.py:26-70 (decay / no-decay groups; layer_scale_* and the custom
                    LayerNorm params fall in no group and are never updated — reproduced)
  FusedAdamW        torch.optim.AdamW(lr, betas=(0.9, 0.999), wd) of train.py:210-216 as one HIP launch
                    per group over flat float32 buffers, also refreshing the bf16 GEMM weight copies
  WarmUpPolyLR      utils/lr_policy.py:22-36
  GradBuckets       DDP-style bucketed gradient all-reduce (SUM, /world folded into AdamW), launched
                    from post-accumulate-grad hooks so RCCL overlaps the rest of the backward pass
  LossScaler        torch.cuda.amp.GradScaler() of the fp16 path (utils/train.py:288-289, 327-337):
                    scaled backward, inf/nan check over the flat gradients on the device, skipped
                    step + backoff on overflow, growth every 2000 clean steps
"""
import torch
import torch.distributed as dist
import torch.nn as nn

from . import kernels as K
from .decoders import collectives_on
from .functional import invalidate_weights, join_streams, register_grad_slot, register_shadow


def group_weight(module, norm_layer=nn.BatchNorm2d):
    """(decay, no_decay) parameter lists exactly as init_func.group_weight builds them."""
    decay, no_decay = [], []
    for m in module.modules():
        if isinstance(m, nn.Linear):
            decay.append(m.weight)
            if m.bias is not None:
                no_decay.append(m.bias)
        elif isinstance(m, (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.ConvTranspose3d)):
            decay.append(m.weight)
            if m.bias is not None:
                no_decay.append(m.bias)
        elif isinstance(m, (norm_layer, nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.GroupNorm, nn.LayerNorm,
                            nn.SyncBatchNorm)):
            if m.weight is not None:
                no_decay.append(m.weight)
            if m.bias is not None:
                no_decay.append(m.bias)
    return decay, no_decay


class WarmUpPolyLR:
    def __init__(self, start_lr, lr_power, total_iters, warmup_steps):
        self.start_lr, self.lr_power = start_lr, lr_power
        self.total_iters, self.warmup_steps = total_iters + 0.0, warmup_steps

    def get_lr(self, cur_iter):
        if cur_iter < self.warmup_steps:
            return self.start_lr * (cur_iter / self.warmup_steps)
        return self.start_lr * ((1 - float(cur_iter) / self.total_iters) ** self.lr_power)


def _chain_order(params, chains):
    """params reordered so that the members of each chain follow its first member (a chain's flat
    slots are then adjacent: one view serves the fused GEMM over them, e.g. q | q_cut | l).
    Only chains whose head is in `params` are regrouped; a member whose head is frozen (or in the
    other group) keeps its own position, so every parameter of `params` lands in the result exactly
    once (the GEMM then falls back to separate slots: gslot_rows / _adjacent_rows return None)."""
    present = {id(p) for p in params}
    follow = {}
    members = set()
    for ch in chains:
        ch = [p for p in ch if p is not None]
        if len(ch) > 1 and id(ch[0]) in present:
            tail = [q for q in ch[1:] if id(q) in present and id(q) not in members]
            follow[id(ch[0])] = tail
            members.update(id(q) for q in tail)
    out, done = [], set()

    def emit(p):  # p, then its chain's tail (a tail member that heads a chain of its own brings that tail)
        if id(p) in done:
            return
        done.add(id(p))
        out.append(p)
        for q in follow.get(id(p), []):
            emit(q)

    for p in params:
        if id(p) not in members:
            emit(p)
    for p in params:  # members reachable from no emitted head (chains that form a cycle)
        emit(p)
    assert len(out) == len(params), "chain reorder lost or duplicated a parameter"
    return out


def fused_chains(model):
    """Parameter chains whose flat slots must be adjacent: each Attention's q | q_cut | l weights
    and biases (one GEMM in the forward, one weight-gradient GEMM in the backward), proj | proj_e,
    and every BatchNorm's bias | weight (the BN backward statistics (sum dy, sum dy * xhat) are
    written straight into them, decoders.bn_grad_stats)."""
    chains = []
    for m in model.modules():
        if isinstance(m, nn.modules.batchnorm._BatchNorm) and m.affine:
            chains.append([m.bias, m.weight])
        if all(hasattr(m, n) for n in ("q", "q_cut", "l", "proj")):
            chains.append([m.q.weight, m.q_cut.weight, m.l.weight])
            chains.append([m.q.bias, m.q_cut.bias, m.l.bias])
            if getattr(m, "proj_e", None) is not None:
                chains.append([m.proj.weight, m.proj_e.weight])
                chains.append([m.proj.bias, m.proj_e.bias])
    return chains


class _FlatGroup:
    """Parameters of one optimizer group re-homed into one flat float32 buffer (+ grad, m, v, bf16)."""

    def __init__(self, params, wd, device, shadow_dtype, chains=()):
        self.params = _chain_order([p for p in params if p.requires_grad], chains)
        self.wd = wd
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, device=device, dtype=torch.float32)
        self.grad = torch.zeros(n, device=device, dtype=torch.float32)
        self.m = torch.zeros(n, device=device, dtype=torch.float32)
        self.v = torch.zeros(n, device=device, dtype=torch.float32)
        self.shadow = torch.empty(n, device=device, dtype=shadow_dtype) if shadow_dtype != torch.float32 else None
        self.slots = {}
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            self.slots[p] = (off, k)
            register_grad_slot(p, self.grad, off)
            off += k
        if self.shadow is not None:
            self.shadow.copy_(self.flat)

    def register_shadows(self):
        if self.shadow is None:
            return
        for p, (off, k) in self.slots.items():
            if p.dim() >= 2:
                register_shadow(p, self.shadow[off:off + k].view(p.shape[0], -1))


class GradBuckets:
    """Copies each parameter's finished gradient into its group's flat buffer; with world > 1 it
    launches an async all-reduce per ~25 MB bucket as soon as the bucket is complete."""

    def __init__(self, groups, world, bucket_bytes=25 << 20):
        self.world = world
        self.handles = []
        self.buckets = []  # (tensor view, set(params))
        self.owner = {}
        for gi, g in enumerate(groups):
            start, cur, members = None, 0, []
            order = sorted(g.slots.items(), key=lambda kv: -kv[1][0])  # reverse registration ~ backward order
            for p, (off, k) in order:
                members.append(p)
                cur += k * 4
                start = off if start is None else min(start, off)
                if cur >= bucket_bytes:
                    self._add(g, members, start)
                    start, cur, members = None, 0, []
            if members:
                self._add(g, members, start)
        self.pending = [len(b[1]) for b in self.buckets]
        self.copies = [[] for _ in self.buckets]
        self.fired = set()  # ids of parameters whose gradient arrived this step
        self.unfired = []  # (group, off, k) of the last finished step's parameters without a gradient
        self.main_stream = None  # the stream the step's backward starts from (set by train_step)
        self.checked = False  # the unused-parameter set was compared across ranks (first step)
        for p in self.owner:
            p.register_post_accumulate_grad_hook(self._hook)

    def _check_unused_consistent(self):
        """The parameters that got no gradient must be the same on every rank: their slots are
        zeroed and their values / moments restored per rank while their bucket is still summed, so
        ranks with different unused sets would silently diverge (the reference's DDP,
        find_unused_parameters=False, raises instead). One small all-reduce of the per-parameter
        fired mask (MAX of [fired, -fired]) on the first step; the model's unused set is static."""
        params = list(self.owner)
        fired = torch.tensor([1.0 if id(p) in self.fired else 0.0 for p in params],
                             device=self.buckets[0][0].device)
        both = torch.cat([fired, -fired])
        dist.all_reduce(both, op=dist.ReduceOp.MAX)
        n = len(params)
        if not torch.equal(both[:n], -both[n:]):  # max(fired) != min(fired) somewhere
            bad = [i for i in range(n) if float(both[i]) != float(-both[n + i])]
            raise RuntimeError(f"ranks disagree on which parameters received gradients ({len(bad)} parameters, "
                               f"e.g. shape {tuple(params[bad[0]].shape)}); DDP with "
                               "find_unused_parameters=False would fail the same way")
        self.checked = True

    def _add(self, g, members, start):
        end = max(g.slots[p][0] + g.slots[p][1] for p in members)
        bi = len(self.buckets)
        self.buckets.append((g.grad[start:end], set(members)))
        for p in members:
            self.owner[p] = (bi, g)

    def _hook(self, p):
        bi, g = self.owner[p]
        off, k = g.slots[p]
        if p.grad.data_ptr() != g.grad.data_ptr() + 4 * off:  # kernels usually wrote the slot directly
            self.copies[bi].append((g.grad[off:off + k], p.grad.reshape(-1)))
        p.grad = None
        self.fired.add(id(p))
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            self._flush(bi)
            # first step: every bucket is reduced in finish(), after the cross-rank unused-set check
            # (a collective issued here on one rank would pair with that check on another)
            if collectives_on(self.world) and self.checked:
                # the bucket mixes slots written on the main stream, the side streams (RGB ConvFFN,
                # attention backward) and the weight-gradient stream, and this hook runs on whichever
                # stream autograd replays the last AccumulateGrad on: wait for all of them before RCCL
                # reads it
                join_streams(self.main_stream)
                self.handles.append(dist.all_reduce(self.buckets[bi][0], async_op=True))

    def _flush(self, bi):
        """Gradients autograd produced outside the slots (torch-managed stems, decoder BN affine
        params): one multi-tensor copy launch per bucket instead of one copy per parameter."""
        pairs = self.copies[bi]
        if pairs:
            torch._foreach_copy_([d for d, _ in pairs], [s for _, s in pairs])
            self.copies[bi] = []

    def finish(self):
        """Join the step's all-reduces. Buckets holding a parameter that got no gradient this step
        (an unused branch) are completed here: the slots of such parameters are zeroed first (they
        still hold the previous step's gradient, and torch's AdamW after zero_grad() would see no
        gradient either), then the bucket is reduced like the others. Their (group, offset, numel)
        are left in `unfired`: torch's AdamW skips a parameter whose .grad is None, so FusedAdamW
        restores their value and moments after its flat update."""
        self.unfired = []
        first = not self.checked
        if collectives_on(self.world) and first:
            self._check_unused_consistent()
        for bi, b in enumerate(self.buckets):
            if self.pending[bi] > 0:
                for p in b[1]:
                    if id(p) not in self.fired:
                        g = self.owner[p][1]
                        off, k = g.slots[p]
                        g.grad[off:off + k].zero_()
                        self.unfired.append((g, off, k))
                self._flush(bi)
            if (self.pending[bi] > 0 or first) and collectives_on(self.world):
                join_streams(self.main_stream)
                self.handles.append(dist.all_reduce(b[0], async_op=True))
        for h in self.handles:
            h.wait()
        self.handles = []
        self.fired = set()
        self.pending = [len(b[1]) for b in self.buckets]


class LossScaler:
    """torch.cuda.amp.GradScaler defaults (init 2**16, growth 2.0, backoff 0.5, interval 2000) for
    the fp16 compute dtype, decided on the device so the fp16 step replays from a captured graph:
    `state` = float32 {scale, growth_tracker, applied_steps, skipped}. The loss gradient is seeded
    with a view of state[0]; the optimizer flags inf / nan in every flat gradient buffer
    (dfm_grad_nonfinite), the AdamW kernels skip the update on overflow and unscale by 1/scale
    otherwise, and dfm_loss_scale_update applies GradScaler.update and clears the flag. Nothing is
    read on the host during a step."""

    def __init__(self, device, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        self.growth_factor, self.backoff_factor, self.growth_interval = growth_factor, backoff_factor, growth_interval
        self.state = torch.tensor([float(init_scale), 0.0, 0.0, 0.0], device=device, dtype=torch.float32)
        self.found_inf = torch.zeros(1, device=device, dtype=torch.int32)

    @property
    def scale(self):
        return float(self.state[0])

    @property
    def growth_tracker(self):
        return int(self.state[1])

    @property
    def skipped(self):
        return int(self.state[3])

    def seed(self, loss):
        """The backward seed scale * d(loss): a view of the device scale, read at replay time."""
        return self.state[0].view(()).expand_as(loss)

    def flag_nonfinite(self, grads):
        for g in grads:
            K.grad_nonfinite(g, self.found_inf)

    def update_device(self):
        K.loss_scale_update(self.state, self.found_inf, self.growth_factor, self.backoff_factor,
                            self.growth_interval)

    def update(self, found_inf):
        """GradScaler.update on the state from the host (what dfm_loss_scale_update does on the
        device; used where no device is involved)."""
        st = self.state
        if found_inf:
            st[0] *= self.backoff_factor
            st[1] = 0.0
            st[3] += 1.0
        else:
            st[2] += 1.0
            st[1] += 1.0
            if st[1] >= self.growth_interval:
                st[0] *= self.growth_factor
                st[1] = 0.0


class FusedAdamW:
    """torch.optim.AdamW semantics over the two group_weight groups (decay wd, no-decay 0).

    One step count for every parameter: torch's AdamW keeps a per-parameter 'step' and does not
    advance it for a parameter without a gradient, whereas here a parameter that was skipped in
    some steps (its value and moments restored, see GradBuckets.finish) still uses the global count
    in the bias correction. DFormer's unused parameters never get a gradient, so this only matters
    for a model whose used set changes between steps."""

    def __init__(self, model, lr=6e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, world=1,
                 compute_dtype=torch.float32, bucket_bytes=25 << 20):
        decay, no_decay = group_weight(model)
        self.full_groups = (decay, no_decay)  # reference group lists, incl. frozen params (state_dict indices)
        dev = next(model.parameters()).device
        chains = fused_chains(model)
        self.groups = [_FlatGroup(decay, weight_decay, dev, compute_dtype, chains),
                       _FlatGroup(no_decay, 0.0, dev, torch.float32, chains)]
        self.lr, self.betas, self.eps = lr, betas, eps
        self.world = world
        # fp16 compute (BASELINE config 5, the reference's --amp): dynamic loss scaling on the device
        self.scaler = LossScaler(dev) if compute_dtype == torch.float16 else None
        self.step_count = 0
        # [lr, step] on the device, read by the AdamW kernel: the same arithmetic whether the step
        # runs eagerly (step() refreshes it) or replays from a captured graph (the graph's owner
        # refreshes it before every replay and sets external_hyper)
        self.hyper = torch.zeros(2, device=dev, dtype=torch.float32)
        self.external_hyper = False
        self.buckets = GradBuckets(self.groups, world, bucket_bytes)
        grouped = {id(p) for g in self.groups for p in g.params}
        # layer_scale_* and the custom LayerNorm params: in no group (never updated, like the reference)
        self.ungrouped = [p for p in model.parameters() if p.requires_grad and id(p) not in grouped]
        invalidate_weights()
        for g in self.groups:
            g.register_shadows()

    @property
    def step_count(self):
        """Applied optimizer steps (torch's AdamW state 'step'). With the fp16 scaler the count lives
        on the device (an overflowing step is skipped there), so reading it synchronises."""
        return int(self.scaler.state[2]) if self.scaler is not None else self._steps

    @step_count.setter
    def step_count(self, v):
        if self.scaler is not None:
            self.scaler.state[2] = float(v)
        else:
            self._steps = v

    def step(self, lr=None):
        join_streams(self.buckets.main_stream)  # every gradient-writing stream is done
        self.buckets.finish()
        for p in self.ungrouped:
            p.grad = None
        gscale = 1.0 / self.world
        sc = self.scaler
        if sc is not None:  # GradScaler.unscale_ / step / update, decided on the device
            sc.flag_nonfinite([g.grad for g in self.groups])
        else:
            self._steps += 1
        lr = self.lr if lr is None else lr
        if not self.external_hyper:
            self.hyper[0].fill_(lr)
            if sc is None:
                self.hyper[1].fill_(float(self._steps))
        # parameters that got no gradient this step: torch.optim.AdamW skips them (no decay, no
        # momentum step), so their value / moments are put back after the flat update
        keep = [(g, off, k, g.flat[off:off + k].clone(), g.m[off:off + k].clone(), g.v[off:off + k].clone())
                for g, off, k in self.buckets.unfired]
        for g in self.groups:
            K.adamw(g.flat, g.grad, g.m, g.v, lr, self.betas[0], self.betas[1], self.eps, g.wd, 1, gscale, g.shadow,
                    hyper=self.hyper, amp=sc.state if sc is not None else None,
                    flag=sc.found_inf if sc is not None else None)
        if sc is not None:
            sc.update_device()
        for g, off, k, p0, m0, v0 in keep:
            g.flat[off:off + k].copy_(p0)
            g.m[off:off + k].copy_(m0)
            g.v[off:off + k].copy_(v0)
            if g.shadow is not None:
                g.shadow[off:off + k].copy_(p0)
        invalidate_weights()
        for g in self.groups:
            g.register_shadows()


    def refresh_shadows(self):
        """After parameters were overwritten in place (load_state_dict): refresh the bf16 copies."""
        for g in self.groups:
            if g.shadow is not None:
                g.shadow.copy_(g.flat)
        invalidate_weights()
        for g in self.groups:
            g.register_shadows()

    # ---- torch.optim.AdamW-compatible state (utils/engine/engine.py:101-186 save/restore)
    def state_dict(self):
        """The state_dict torch.optim.AdamW over group_weight's two groups would have: parameters
        indexed in group order (frozen ones included, without state), exp_avg / exp_avg_sq / step."""
        defaults = {k: v for k, v in torch.optim.AdamW([torch.zeros(1, requires_grad=True)]).param_groups[0].items()
                    if k != "params"}
        state, groups, idx = {}, [], 0
        steps = self.step_count  # one read (a device sync with the fp16 scaler), not one per parameter
        for plist, g in zip(self.full_groups, self.groups):
            ids = []
            for p in plist:
                if p in g.slots and steps > 0:
                    off, k = g.slots[p]
                    state[idx] = {"step": torch.tensor(float(steps)),
                                  "exp_avg": g.m[off:off + k].view_as(p).detach().clone(),
                                  "exp_avg_sq": g.v[off:off + k].view_as(p).detach().clone()}
                ids.append(idx)
                idx += 1
            grp = dict(defaults)
            grp.update(lr=self.lr, betas=self.betas, eps=self.eps, weight_decay=g.wd, params=ids)
            groups.append(grp)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        groups = sd["param_groups"]
        if len(groups) != 2:
            raise ValueError(f"expected the two group_weight groups, got {len(groups)}")
        steps = set()
        for plist, g, grp in zip(self.full_groups, self.groups, groups):
            if len(grp["params"]) != len(plist):
                raise ValueError(f"param group size mismatch: {len(grp['params'])} vs {len(plist)}")
            for p, idx in zip(plist, grp["params"]):
                st = sd["state"].get(idx, sd["state"].get(str(idx)))
                if st is None or p not in g.slots:
                    continue
                off, k = g.slots[p]
                g.m[off:off + k].copy_(st["exp_avg"].reshape(-1))
                g.v[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(float(st["step"])))
        self.lr = groups[0].get("lr", self.lr)
        self.betas = tuple(groups[0].get("betas", self.betas))
        self.eps = groups[0].get("eps", self.eps)
        if len(steps) > 1:
            raise ValueError(f"per-parameter step counts differ: {sorted(steps)[:4]}")
        self.step_count = steps.pop() if steps else 0


def all_reduce_mean(t, world):
    """pyt_utils.all_reduce_tensor (SUM then /world), async-free for the scalar loss."""
    if collectives_on(world):
        t = t.clone()
        dist.all_reduce(t)
        t = t / world
    return t


class GraphedTrainStep:
    """train_step captured once into a HIP graph (torch.cuda.graph) and replayed: the whole
    forward + loss + backward + AdamW step of ~2.3k kernel launches becomes one graph launch, so
    the host (~23 us of Python / autograd per eager launch) no longer paces the device.

    rgb / depth / label are the static input buffers: copy each new batch into them in place. The
    optimizer's lr and step count live in a device tensor refreshed before every replay (the only
    per-step host state of the step); dropout / DropPath draws advance with torch's graph-safe
    Philox offsets. Needs every kernel of the step on torch's current stream or streams forked from
    it (true of this package) and no host synchronisation inside the step."""

    def __init__(self, model, opt, rgb, depth, label, warmup=2):
        self.model, self.opt = model, opt
        self.inputs = (rgb, depth, label)
        side = torch.cuda.Stream(device=rgb.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up on a side stream, as torch.cuda.graph requires
            for _ in range(warmup):
                train_step(model, opt, rgb, depth, label)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if collectives_on(opt.world) and dist.get_backend() == "nccl":
            # the RCCL watchdog thread polls the events of the warm-up's collectives until it retires
            # them; a poll failing under the capture makes it rethrow on its own thread (SIGABRT seen
            # once in capture_end): nothing of the eager steps may still be pending when capture begins
            dist.distributed_c10d._get_default_group()._wait_for_pending_works()
        self.graph = torch.cuda.CUDAGraph()
        opt.external_hyper = True  # inside the graph AdamW only reads hyper
        try:
            # thread-local capture: the process group's watchdog thread keeps querying the events of
            # earlier (eager) collectives, which under the default global mode invalidates the capture
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self.loss = train_step(model, opt, rgb, depth, label)  # host step_count advanced once here
        finally:
            opt.external_hyper = False

    def _set_hyper(self, lr, step):
        self.opt.hyper[0].fill_(self.opt.lr if lr is None else lr)
        if step is not None:
            self.opt.hyper[1].fill_(float(step))

    def __call__(self, lr=None):
        """One training step (the first call replays the captured step itself)."""
        amp = self.opt.scaler is not None  # the fp16 step counts its applied steps on the device
        if getattr(self, "_replayed", False) and not amp:
            self.opt._steps += 1
        self._replayed = True
        self._set_hyper(lr, None if amp else self.opt._steps)
        self.graph.replay()
        return self.loss

    def eager(self, lr=None):
        """One step issued from Python on the same model / optimizer / inputs (probe windows)."""
        return train_step(self.model, self.opt, *self.inputs, lr=lr)


def train_step(model, opt, rgb, depth, label, lr=None):
    """One reference training iteration (train.py:318-357): forward + loss, backward (bucketed
    RCCL all-reduce overlapping it), loss all-reduce, AdamW step. Returns the (device) mean loss."""
    loss, _ = model(rgb, depth, label)
    reduce_loss = all_reduce_mean(loss.detach(), opt.world)
    opt.buckets.main_stream = torch.cuda.current_stream() if loss.is_cuda else None
    if opt.scaler is not None:  # scaler.scale(loss).backward(), the scale read on the device
        loss.backward(opt.scaler.seed(loss))
    else:
        loss.backward()
    opt.step(lr)
    return reduce_loss
