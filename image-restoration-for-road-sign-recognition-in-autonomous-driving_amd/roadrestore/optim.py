"""Fused Adam / AdamW (one HIP launch per contiguous parameter span).

Update rule = torch.optim.Adam / AdamW (the reference's optimisers, 07:143 and
14:222): decoupled weight decay p *= 1 - lr*wd (AdamW), m.lerp_(g, 1-b1),
v = b2 v + (1-b2) g^2, p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).

When the parameters (``flatten_parameters``) and their gradients (written by
the network's backward into one flat buffer in the same order) each tile one
contiguous span, a step is a single kernel over every parameter; otherwise
one launch per parameter.  The learning-rate schedule is host arithmetic:
torch.optim.lr_scheduler.CosineAnnealingLR works unchanged (14:223, 248).

``capturable=True`` (HIP-graph replay of the whole step): the step count AND
the learning rate live on the device.  Each group's ``lr`` becomes ONE
persistent 1-element fp32 device tensor; torch's LR schedulers update a tensor
lr in place (``fill_``), which the captured ``rr_adamw_dev`` launch reads on
every replay, so ``scheduler.step()`` between replays takes effect.  Only
in-place updates reach a replay: a plain ``group["lr"] = x`` (warm-up code)
swaps the tensor out of the group, and the graph keeps reading the old one.
The next eager ``step()`` (or capture) copies such a value back into the
persistent tensor, with a warning once a graph has been captured.
``state_dict()`` reports lr as a Python float.
"""
from __future__ import annotations

import warnings

import torch

from . import ops
from ._lib import lib

CosineAnnealingLR = torch.optim.lr_scheduler.CosineAnnealingLR

# global parameter generation: incremented by every fused optimizer step
# (engine.WeightCache keys on it in addition to the tensor version counters)
GENERATION = [0]


def _bump_versions(tensors):
    GENERATION[0] += 1
    inc = getattr(torch.autograd.graph, "increment_version", None)
    if inc is not None:
        inc(tensors)


def flatten_parameters(model, order=None):
    """Re-home ``model``'s parameters into one contiguous fp32 buffer laid out
    in ``order`` (default: the network's gradient layout), so the fused
    optimiser updates all of them with one launch.  Values are preserved."""
    if order is None:
        order = model.grad_layout() if hasattr(model, "grad_layout") else list(model.parameters())
    total = sum(p.numel() for p in order)
    dev = order[0].device
    flat = torch.empty(total, dtype=torch.float32, device=dev)
    off = 0
    with torch.no_grad():
        for p in order:
            n = p.numel()
            flat[off:off + n].copy_(p.detach().reshape(-1))
            p.data = flat[off:off + n].view(p.shape)
            off += n
    model._rr_flat_params = flat
    return flat


def _span(tensors):
    """Sorted [(ptr, tensor)] if the tensors tile one contiguous fp32 span."""
    if not tensors:
        return None
    items = sorted(((t.data_ptr(), i) for i, t in enumerate(tensors)))
    exp = items[0][0]
    for ptr, i in items:
        t = tensors[i]
        if ptr != exp or not t.is_contiguous() or t.dtype != torch.float32:
            return None
        exp += t.numel() * 4
    return items


class _FusedAdamBase(torch.optim.Optimizer):
    decoupled = True

    def __init__(self, params, lr, betas, eps, weight_decay, capturable=False):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._gstate = {}
        # capturable: the step count and the learning rate live on the device
        # (rr_adamw_dev) so a HIP-graph replay of optimizer.step() advances the
        # bias correction and follows the LR schedule
        self.capturable = capturable
        if capturable:
            for gi, group in enumerate(self.param_groups):
                self._lr_to_device(gi, group, warn=False)

    def _lr_to_device(self, gi, group, warn=True):
        """The group's persistent 1-element fp32 lr tensor on the parameters'
        device (once they are on a GPU), holding group["lr"]'s value; put back
        into the group if it was replaced.  Returns it or None."""
        dev = next((p.device for p in group["params"] if p.is_cuda), None)
        if dev is None:
            return None
        gstate = self._gstate.setdefault(gi, {})
        lr_t = gstate.get("lr_dev")
        lr = group["lr"]
        if lr_t is None or lr_t.device != dev:
            lr_t = torch.empty(1, dtype=torch.float32, device=dev)
            lr_t.fill_(float(lr))
            gstate["lr_dev"] = lr_t
        elif lr is not lr_t:
            if warn and gstate.get("captured"):
                warnings.warn("param_groups[%d]['lr'] was replaced after a HIP-graph capture: "
                              "graph replays keep reading the persistent lr tensor; update it "
                              "in place (group['lr'].fill_(x)) between replays" % gi)
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("param_groups[%d]['lr'] was replaced; it cannot be copied to "
                                   "the device during a capture" % gi)
            lr_t.fill_(float(lr))
        group["lr"] = lr_t
        return lr_t

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        if self.capturable:
            for gi, group in enumerate(self.param_groups):
                self._lr_to_device(gi, group, warn=False)

    def state_dict(self):
        sd = super().state_dict()
        for g in sd["param_groups"]:
            if isinstance(g.get("lr"), torch.Tensor):
                g["lr"] = float(g["lr"].item())
        return sd

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            if any(not p.is_cuda for p in ps):
                raise RuntimeError("fused Adam/AdamW runs on the GPU only")
            b1, b2 = group["betas"]
            gi = self.param_groups.index(group)
            gstate = self._gstate.setdefault(gi, {})
            gstate["step"] = gstate.get("step", 0) + 1
            step = gstate["step"]
            pspan = _span([p.data for p in ps])
            gspan = _span([p.grad for p in ps]) if pspan is not None else None
            flat_ok = (pspan is not None and gspan is not None and
                       [i for _, i in pspan] == [i for _, i in gspan])
            if flat_ok:
                key = tuple(id(ps[i]) for _, i in pspan)
                if gstate.get("key") != key:
                    total = sum(p.numel() for p in ps)
                    gstate["m"] = torch.zeros(total, dtype=torch.float32, device=ps[0].device)
                    gstate["v"] = torch.zeros_like(gstate["m"])
                    gstate["key"] = key
                    off = 0
                    for _, i in pspan:
                        p = ps[i]
                        st = self.state.setdefault(p, {})
                        st["exp_avg"] = gstate["m"][off:off + p.numel()].view(p.shape)
                        st["exp_avg_sq"] = gstate["v"][off:off + p.numel()].view(p.shape)
                        off += p.numel()
                total = gstate["m"].numel()
                if self.capturable:
                    if "step_dev" not in gstate:
                        gstate["step_dev"] = torch.full((1,), step - 1, dtype=torch.int64,
                                                        device=ps[0].device)
                    lr_dev = self._lr_to_device(gi, group)
                    if torch.cuda.is_current_stream_capturing():
                        gstate["captured"] = True
                    lib().check(lib().rr_adamw_dev(
                        total, pspan[0][0], gspan[0][0], gstate["m"].data_ptr(),
                        gstate["v"].data_ptr(), lr_dev.data_ptr(), float(b1), float(b2),
                        float(group["eps"]), float(group["weight_decay"]), int(self.decoupled),
                        gstate["step_dev"].data_ptr(), ops.stream()), "rr_adamw_dev")
                else:
                    lib().check(lib().rr_adamw(total, pspan[0][0], gspan[0][0],
                                               gstate["m"].data_ptr(), gstate["v"].data_ptr(),
                                               float(group["lr"]), float(b1), float(b2),
                                               float(group["eps"]), float(group["weight_decay"]),
                                               int(self.decoupled), step, ops.stream()), "rr_adamw")
            else:
                if self.capturable:
                    raise RuntimeError("capturable Adam/AdamW needs flattened parameters "
                                       "(roadrestore.optim.flatten_parameters)")
                for p in ps:
                    st = self.state.setdefault(p, {})
                    if "exp_avg" not in st:
                        st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                        st["exp_avg_sq"] = torch.zeros_like(st["exp_avg"])
                    ops.adamw_(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"],
                               group["lr"], b1, b2, group["eps"], group["weight_decay"],
                               self.decoupled, step)
            for p in ps:
                self.state.setdefault(p, {})["step"] = step
            # the fused kernel wrote through raw pointers: bump the version
            # counters so packed-weight caches (engine.WeightCache) and autograd
            # see the in-place update
            _bump_versions([p.data for p in ps])
        return loss


class AdamW(_FusedAdamBase):
    """torch.optim.AdamW semantics (14:222: lr 2e-4, wd 1e-4)."""

    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 capturable=False):
        super().__init__(params, lr, betas, eps, weight_decay, capturable)


class Adam(_FusedAdamBase):
    """torch.optim.Adam semantics (07:143: lr 1e-3, L2 weight decay folded into g)."""

    decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 capturable=False):
        super().__init__(params, lr, betas, eps, weight_decay, capturable)


class RunningLoss:
    """Device-side running loss: ``add(loss)`` is one asynchronous launch
    (rr_scalar_accumulate), replacing the reference's per-step
    ``running_loss += loss.item()`` (14:246), which synchronises the host with
    the GPU every step.  ``mean()`` / ``total()`` synchronise once (per epoch);
    ``reset()`` starts a new epoch.  Capturable in a HIP graph."""

    def __init__(self, device=None):
        from . import ops
        self._ops = ops
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.acc = torch.zeros(1, dtype=torch.float64, device=dev)
        self.count = torch.zeros(1, dtype=torch.int64, device=dev)

    def add(self, loss):
        from ._lib import lib
        if loss.dtype != torch.float32 or loss.numel() != 1 or not loss.is_cuda:
            raise TypeError("RunningLoss.add expects a 1-element fp32 device tensor")
        lib().check(lib().rr_scalar_accumulate(loss.data_ptr(), self.acc.data_ptr(),
                                               self.count.data_ptr(), self._ops.stream()),
                    "rr_scalar_accumulate")

    def total(self):
        return self.acc.item()

    def steps(self):
        return int(self.count.item())

    def mean(self):
        n = self.steps()
        return self.acc.item() / n if n else float("nan")

    def reset(self):
        self._ops.zero_(self.acc)
        self._ops.zero_(self.count)
