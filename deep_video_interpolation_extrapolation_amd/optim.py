"""Adamax on libdvie (reference optimizer: torch.optim.Adamax, runners/InterTrainer.py:79).

Same constructor, param_groups and state_dict layout as torch.optim.Adamax (per-parameter
state {'step', 'exp_avg', 'exp_inf'}), so checkpoints interchange.  When a group's
parameters are exactly the views of one FlatParams buffer (the HRNet case) and their
.grad tensors are views of its flat gradient, the whole group updates in ONE fused HIP
kernel over the flat buffers (state tensors are views of two flat state buffers);
otherwise one fused-kernel launch per parameter.
"""
import torch

from . import _lib as L


class Adamax(torch.optim.Optimizer):
    def __init__(self, params, lr=2e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._flat = {}

    def _flat_group(self, gi, group):
        """(owner, flat state m, flat state u) if the group maps onto one flat buffer."""
        ps = group["params"]
        owner = getattr(ps[0], "_dvie_owner", None) if ps else None
        if owner is None or any(getattr(p, "_dvie_owner", None) is not owner for p in ps):
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
        ent = self._flat.get(gi)
        if ent is None or ent[1].device != flat.device or ent[1].numel() != flat.numel():
            m = torch.zeros_like(flat)
            u = torch.zeros_like(flat)
            for p in ps:
                off = (p.data_ptr() - flat.data_ptr()) // 4
                st = self.state[p]
                if "exp_avg" in st:  # e.g. after load_state_dict
                    m[off:off + p.numel()].copy_(st["exp_avg"].reshape(-1))
                    u[off:off + p.numel()].copy_(st["exp_inf"].reshape(-1))
                st["exp_avg"] = m[off:off + p.numel()].view_as(p)
                st["exp_inf"] = u[off:off + p.numel()].view_as(p)
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
        lib = L.load()
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            eps, wd, lr = group["eps"], group["weight_decay"], group["lr"]
            flat = self._flat_group(gi, group)
            if flat is not None:
                owner, m, u = flat
                ps = group["params"]
                st0 = self.state[ps[0]]
                step = float(st0["step"]) + 1
                for p in ps:
                    self.state[p]["step"] = torch.tensor(step)
                clr = lr / (1 - b1 ** step)
                L.check(lib.dvie_adamax(owner._flat.data_ptr(), owner._flat_grad.data_ptr(), m.data_ptr(),
                                        u.data_ptr(), owner._flat.numel(), clr, b1, b2, eps, wd,
                                        L.stream_ptr(owner._flat.device)), "adamax")
                continue
            for p in group["params"]:
                if p.grad is None:
                    continue
                L.require_gpu(p)
                st = self.state[p]
                if len(st) == 0 or "exp_avg" not in st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_inf"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                clr = lr / (1 - b1 ** float(st["step"]))
                g = p.grad.contiguous()
                assert p.is_contiguous() and st["exp_avg"].is_contiguous()
                L.check(lib.dvie_adamax(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                        st["exp_inf"].data_ptr(), p.numel(), clr, b1, b2, eps, wd,
                                        L.stream_ptr(p.device)), "adamax")
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat = {}  # re-bind flat state views (copies loaded values in _flat_group)
