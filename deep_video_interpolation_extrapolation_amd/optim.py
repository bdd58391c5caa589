"""Fused optimizers on libdvie.

* `Adamax`: the generator optimizer (torch.optim.Adamax, runners/InterTrainer.py:79).
* `Adam`: the discriminator optimizers (torch.optim.Adam, runners/InterGANTrainer.py:110-112),
  torch 1.0.1 update form (eps added to sqrt(v) before the bias-correction scaling).

Same constructors, param_groups and state_dict layouts as torch.optim (per-parameter state
{'step', 'exp_avg', 'exp_inf'} / {'step', 'exp_avg', 'exp_avg_sq'}), so checkpoints
interchange.  When a group's parameters are exactly the views of one FlatParams buffer
(HRNet, the discriminators) and their .grad tensors are views of its flat gradient, the
whole group updates in ONE fused HIP kernel over the flat buffers (state tensors are views
of two flat state buffers); otherwise one fused-kernel launch per parameter.
"""
import math

import torch

from . import _lib as L



def _owner(p):
    """the FlatParams module whose flat buffer holds parameter p (runtime.FlatParams keeps a
    weak reference on the parameter), or None"""
    r = getattr(p, "_dvie_owner", None)
    return r() if r is not None else None

class _FusedOptimizer(torch.optim.Optimizer):
    STATE = ("exp_avg", "exp_inf")

    def __init__(self, params, lr, betas, eps, weight_decay):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._flat = {}
        self.capturable = False
        self._dsteps = {}
        self._split = {}  # capturable: group index -> per-parameter step counts differ

    def _launch(self, p, g, s0, s1, n, group, step, device):
        raise NotImplementedError

    def _launch_dev(self, p, g, s0, s1, n, group, dstep, device):
        raise NotImplementedError

    def set_capturable(self, flag=True):
        """Graph capture (runners/graph.py): keep every step count on the device and
        compute the bias correction there, so a captured step replays correctly.  The
        first step after switching must run eagerly (it moves the counts)."""
        self.capturable = bool(flag)
        if not flag:
            for st in self.state.values():
                if "step" in st and torch.is_tensor(st["step"]) and st["step"].is_cuda:
                    st["step"] = st["step"].detach().cpu().clone()
            self._dsteps = {}
        self._split = {}

    def _dev_step(self, key, params, device):
        """one device step tensor shared by `params` (created from their host count)"""
        d = self._dsteps.get(key)
        if d is None or d.device != device:
            if torch.cuda.is_current_stream_capturing():
                # a count created here would be re-initialised by every replay
                raise RuntimeError("capturable optimizer: a parameter takes its first step inside the captured "
                                   "step (e.g. SpectralNorm u / v, trainable from the second step): run more "
                                   "eager warm-up steps before capturing")
            st = self.state[params[0]]
            d = torch.full((1,), float(st.get("step", 0.0)), dtype=torch.float32, device=device)
            self._dsteps[key] = d
        for p in params:
            self.state[p]["step"] = d
        return d

    def _host_counts_differ(self, ps):
        counts = set()
        for p in ps:
            st = self.state[p].get("step", 0.0)
            counts.add(float(st.cpu()) if torch.is_tensor(st) else float(st))
        return len(counts) > 1

    def _counts_differ(self, gi, ps):
        """Whether the group's parameters carry different step counts.  Eager: checked on
        the host counts every step.  Capturable: decided on the host counts by the first
        eager step after set_capturable (whether or not every parameter had a gradient then,
        see step()) and kept -- counts that differ once keep differing by the same lag, and a
        captured step must not read device counts back."""
        if self.capturable and gi in self._split:
            return self._split[gi]
        if self.capturable and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("capturable optimizer: run one eager step after set_capturable(True) "
                               "before capturing a step")
        differ = self._host_counts_differ(ps)
        if self.capturable:
            self._split[gi] = differ
        return differ

    def _flat_group(self, gi, group):
        """(owner, flat state 0, flat state 1) if the group maps onto one flat buffer."""
        ps = group["params"]
        owner = _owner(ps[0]) if ps else None
        if owner is None or any(_owner(p) is not owner for p in ps):
            return None
        flat = owner._flat
        if sum(p.numel() for p in ps) != flat.numel():
            return None
        fg = owner._flat_grad
        if fg is None:
            return None
        for p in ps:
            g = p.grad
            if g is None or g.data_ptr() != fg.data_ptr() + (p.data_ptr() - flat.data_ptr()):
                return None
        if self._counts_differ(gi, ps):
            return None  # per-parameter step counts differ (SN u, v become trainable after step 1)
        k0, k1 = self.STATE
        ent = self._flat.get(gi)
        if ent is None or ent[1].device != flat.device or ent[1].numel() != flat.numel():
            m = torch.zeros_like(flat)
            u = torch.zeros_like(flat)
            for p in ps:
                off = (p.data_ptr() - flat.data_ptr()) // 4
                st = self.state[p]
                if k0 in st:  # e.g. after load_state_dict
                    m[off:off + p.numel()].copy_(st[k0].reshape(-1))
                    u[off:off + p.numel()].copy_(st[k1].reshape(-1))
                st[k0] = m[off:off + p.numel()].view_as(p)
                st[k1] = u[off:off + p.numel()].view_as(p)
                st.setdefault("step", torch.tensor(0.0))
            ent = (owner, m, u)
            self._flat[gi] = ent
        return ent

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        k0, k1 = self.STATE
        for gi, group in enumerate(self.param_groups):
            flat = self._flat_group(gi, group)
            if flat is not None and self.capturable:
                owner, m, u = flat
                lib, s = L.load(), L.stream_ptr(owner._flat.device)
                dstep = self._dev_step(("g", gi), group["params"], owner._flat.device)
                L.check(lib.dvie_step_inc(dstep.data_ptr(), s), "step count")
                self._launch_dev(owner._flat, owner._flat_grad, m, u, owner._flat.numel(), group, dstep,
                                 owner._flat.device)
                continue
            if flat is not None:
                owner, m, u = flat
                ps = group["params"]
                step = float(self.state[ps[0]]["step"]) + 1
                for p in ps:
                    self.state[p]["step"] = torch.tensor(step)
                self._launch(owner._flat, owner._flat_grad, m, u, owner._flat.numel(), group, step,
                             owner._flat.device)
                continue
            for p in group["params"]:
                if p.grad is None:
                    continue
                L.require_gpu(p)
                st = self.state[p]
                if len(st) == 0 or k0 not in st:
                    st["step"] = torch.tensor(0.0)
                    st[k0] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st[k1] = torch.zeros_like(p, memory_format=torch.preserve_format)
                g = p.grad.contiguous()
                assert p.is_contiguous() and st[k0].is_contiguous()
                if self.capturable:
                    dstep = self._dev_step(("p", id(p)), [p], p.device)
                    L.check(L.load().dvie_step_inc(dstep.data_ptr(), L.stream_ptr(p.device)), "step count")
                    self._launch_dev(p, g, st[k0], st[k1], p.numel(), group, dstep, p.device)
                    continue
                st["step"] += 1
                self._launch(p, g, st[k0], st[k1], p.numel(), group, float(st["step"]), p.device)
        if self.capturable and not torch.cuda.is_current_stream_capturing():
            # decide every group's split after this eager step, also for a group whose
            # parameters were not all stepped (e.g. SpectralNorm u / v without gradients yet),
            # so that the captured step never reads the step counts back
            for gi, group in enumerate(self.param_groups):
                if gi not in self._split:
                    self._split[gi] = self._host_counts_differ(group["params"])
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat = {}  # re-bind flat state views (copies loaded values in _flat_group)
        self._dsteps = {}
        self._split = {}


class Adamax(_FusedOptimizer):
    STATE = ("exp_avg", "exp_inf")

    def __init__(self, params, lr=2e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        super().__init__(params, lr, betas, eps, weight_decay)

    def _launch(self, p, g, s0, s1, n, group, step, device):
        b1, b2 = group["betas"]
        clr = group["lr"] / (1 - b1 ** step)
        L.check(L.load().dvie_adamax(p.data_ptr(), g.data_ptr(), s0.data_ptr(), s1.data_ptr(), n, clr, b1, b2,
                                     group["eps"], group["weight_decay"], L.stream_ptr(device)), "adamax")

    def _launch_dev(self, p, g, s0, s1, n, group, dstep, device):
        b1, b2 = group["betas"]
        L.check(L.load().dvie_adamax_dev(p.data_ptr(), g.data_ptr(), s0.data_ptr(), s1.data_ptr(), n, group["lr"], b1,
                                         b2, group["eps"], group["weight_decay"], dstep.data_ptr(),
                                         L.stream_ptr(device)), "adamax")


class Adam(_FusedOptimizer):
    STATE = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("amsgrad (unused by the reference)")
        super().__init__(params, lr, betas, eps, weight_decay)

    def _launch(self, p, g, s0, s1, n, group, step, device):
        b1, b2 = group["betas"]
        step_size = group["lr"] * math.sqrt(1 - b2 ** step) / (1 - b1 ** step)
        L.check(L.load().dvie_adam(p.data_ptr(), g.data_ptr(), s0.data_ptr(), s1.data_ptr(), n, step_size, b1, b2,
                                   group["eps"], group["weight_decay"], L.stream_ptr(device)), "adam")

    def _launch_dev(self, p, g, s0, s1, n, group, dstep, device):
        b1, b2 = group["betas"]
        L.check(L.load().dvie_adam_dev(p.data_ptr(), g.data_ptr(), s0.data_ptr(), s1.data_ptr(), n, group["lr"], b1, b2,
                                       group["eps"], group["weight_decay"], dstep.data_ptr(), L.stream_ptr(device)),
                "adam")
