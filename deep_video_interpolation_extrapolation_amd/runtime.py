"""Autograd bridge and parameter storage for plan-executed networks.

* `FlatParams`: every parameter of a module becomes a view into one flat fp32 buffer
  (and its .grad a view into one flat fp32 gradient buffer), laid out in the order the
  backward pass finishes them.  The fused Adamax step and the data-parallel gradient
  all-reduce each then touch one contiguous buffer.
* `PlanFunction`: a torch.autograd.Function whose forward runs a compiled Plan's
  forward op list and whose backward runs its backward op list.  Parameter gradients
  are written straight into the parameters' .grad views by the plan's weight reductions
  (so autograd returns None for them); input gradients are returned as tensors.
* `PlanPool`: plans are cached per (shape, dtype, device, training); a plan whose saved
  activations are still needed by a pending backward is marked busy and a second plan
  is built for any further forward.
"""
import weakref

import torch

from . import _lib as L


def precision_of(args=None, default="fp32"):
    import os
    p = getattr(args, "precision", None) if args is not None else None
    p = p or os.environ.get("DVIE_PRECISION", default)
    if p in ("bf16", "bfloat16"):
        return torch.bfloat16
    if p in ("fp32", "float32", "f32"):
        return torch.float32
    raise ValueError(f"unknown precision {p}")


class FlatParams:
    """Mixin for nn.Modules whose parameters live in one flat buffer."""

    def _flatten(self, order=None):
        params = [p for p in self.parameters()]
        if order is not None:
            idx = {id(p): i for i, p in enumerate(params)}
            ordered = [p for p in order if id(p) in idx]
            seen = {id(p) for p in ordered}
            params = ordered + [p for p in params if id(p) not in seen]
        total = sum(p.numel() for p in params)
        dev = params[0].device if params else torch.device("cpu")
        flat = torch.empty(total, dtype=torch.float32, device=dev)
        specs = []
        off = 0
        for p in params:
            n = p.numel()
            flat[off:off + n].copy_(p.detach().reshape(-1))
            specs.append((off, n, tuple(p.shape)))
            off += n
        for p in params:
            # lets optim.Adamax take the one-launch flat path; a weak reference, so that the
            # module -> plan -> layer -> parameter -> module loop holds no strong edge back to
            # the module (torch does not traverse a tensor's __dict__ for the cycle collector
            # while C++ also refers to the tensor: such a loop kept whole plans -- 100+ GB
            # at 1024x2048 -- alive after their model was deleted)
            p._dvie_owner = weakref.ref(self)
        self._flat_params = params
        self._flat_specs = specs
        self._flat = flat
        self._flat_grad = None
        self._repoint()

    def _repoint(self):
        for p, (off, n, shape) in zip(self._flat_params, self._flat_specs):
            p.data = self._flat[off:off + n].view(shape)

    def flat_grad(self):
        if self._flat_grad is None or self._flat_grad.device != self._flat.device:
            self._flat_grad = torch.zeros_like(self._flat)
        return self._flat_grad

    def grad_views(self, params=None):
        """Attach .grad of every parameter (or of the subset `params`: the ones one plan
        writes, when several plans share the flat buffer) to its view of the flat gradient
        buffer.  Returns True if those parameters already had gradients (accumulate mode)."""
        fg = self.flat_grad()
        accumulate = False
        sel = None if params is None else {id(p) for p in params}
        for p, (off, n, shape) in zip(self._flat_params, self._flat_specs):
            if not p.requires_grad:  # frozen (e.g. SpectralNorm u, v): .grad stays None
                continue
            if sel is not None and id(p) not in sel:
                continue
            if p.grad is None:
                p.grad = fg[off:off + n].view(shape)
            else:
                accumulate = True
        return accumulate

    def _apply(self, fn, recurse=True):
        # move/convert the flat buffer once and re-point every parameter view
        for m in self.modules():  # module buffers (e.g. BatchNorm statistics)
            for k, b in m._buffers.items():
                if b is not None:
                    m._buffers[k] = fn(b)
        new = fn(self._flat)
        self._flat = new
        self._flat_grad = None
        for p, (off, n, shape) in zip(self._flat_params, self._flat_specs):
            p.data = self._flat[off:off + n].view(shape)
            p.grad = None
        self._on_moved()
        return self

    def _on_moved(self):
        pass


class PlanPool:
    def __init__(self, build):
        self.build = build  # key -> Plan
        self.plans = {}

    def acquire(self, key):
        lst = self.plans.setdefault(key, [])
        for p in lst:
            if not p.busy:
                return p
        p = self.build(key)
        lst.append(p)
        return p

    def clear(self):
        self.plans = {}


class _Token:
    """Holds a plan busy until the autograd graph that needs its activations dies."""

    def __init__(self, plan):
        self.plan = plan
        plan.busy = True
        self._fin = weakref.finalize(self, _release, plan)


def _release(plan):
    plan.busy = False


class PlanFunction(torch.autograd.Function):
    """outputs = plan.forward(inputs); backward -> input grads (+ param .grad writes).

    Arguments: (runner, n_inputs, *inputs, *params) — `runner` implements
    `forward(plan_inputs) -> (plan, outputs)` and `backward(plan, grads) -> input grads`.
    """

    @classmethod
    def apply(cls, runner, n_in, *args):
        # ctx.needs_input_grad reports requires_grad even under torch.no_grad(), and grad
        # mode is always off inside forward: record the caller's mode, so an inference
        # forward compiles (and allocates) no backward
        runner._grad_mode = torch.is_grad_enabled()
        return super().apply(runner, n_in, *args)

    @staticmethod
    def forward(ctx, runner, n_in, *args):
        inputs = args[:n_in]
        runner._in_needs = tuple(ctx.needs_input_grad[2:2 + n_in])  # which inputs want a gradient
        train = getattr(runner, "_grad_mode", True) and any(ctx.needs_input_grad)
        plan, outs = runner.run_forward(inputs, train)
        ctx.runner = runner
        ctx.token = _Token(plan) if plan is not None and plan.backward_enabled else None
        ctx.n_in = n_in
        ctx.n_params = len(args) - n_in
        ctx.save_for_backward(*inputs)
        ctx.gen = plan.generation if plan is not None else None
        ctx.mark_non_differentiable(*[o for o in outs if not o.is_floating_point()])
        return tuple(outs) if len(outs) > 1 else outs[0]

    @staticmethod
    def backward(ctx, *grads):
        plan = ctx.token.plan if ctx.token is not None else None
        if plan is None:
            raise RuntimeError("backward through a plan compiled without gradients")
        if plan.generation != ctx.gen:
            raise RuntimeError("plan activations were overwritten before backward")
        inputs = ctx.saved_tensors
        # parameters get a gradient only if they required one at the forward (autograd's rule:
        # a later requires_grad_(True) does not reach back into this graph)
        # (read by runners during this call only: cleared afterwards, so a later run_backward
        # outside PlanFunction never sees this graph's flags)
        ctx.runner._param_needs = tuple(ctx.needs_input_grad[2 + ctx.n_in:])
        try:
            in_grads = ctx.runner.run_backward(plan, inputs, grads, ctx.needs_input_grad[2:2 + ctx.n_in])
        finally:
            ctx.runner._param_needs = None
        plan.busy = False
        ctx.token = None
        return (None, None) + tuple(in_grads) + (None,) * ctx.n_params
