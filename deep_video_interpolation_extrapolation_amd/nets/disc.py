"""Frame / video discriminators of InterGANNet on the MI355X plan engine.

Module trees, construction order (so seeded initialisation) and state_dict keys are those
of the reference:
  FrameDiscriminator nets/FrameDisc.py:35-75, FrameLocalDiscriminator l.77-114,
  FrameSNDiscriminator l.116-156, FrameSNLocalDiscriminator l.158-189,
  VideoDiscriminator nets/VidDisc.py:34-84, VideoLocalDiscriminator l.86-138,
  VideoSNDiscriminator l.140-183, VideoSNLocalDiscriminator l.185-226,
  ResnetBlock / ResnetSNBlock FrameDisc.py:8-32, SpectralNorm nets/SpectralNorm.py:14-68.
The forward and backward do not run the submodules: `_lower` turns `self.layer` into one
engine plan (HIP convs with fused bias / residual / LeakyReLU epilogues, BatchNorm with batch
statistics fused with its LeakyReLU, the AvgPool + view(-1, C).mean(1) head, or, for the
local variants, the last conv writing the (B, 1, h, w) map).  SpectralNorm layers get their
power iteration in one HIP launch before the plan packs the weights (dvie_sn_fwd) and their
sigma adjoint in one launch after its backward (dvie_sn_bwd).

Calling conventions follow the reference: Frame*(x, seg, bboxes=None) and
Video*(x, seg, input_x, input_seg, bboxes=None) -> (B*k,) scores (k pooled cells; k = 1 at
the reference's 128x128 training crops) or the (B, 1, h, w) map of the local variants.  The
input concat (`torch.cat` in the reference forward) is never materialised: each input is
packed into its own channel slice of the first conv's input buffer.
"""
import ctypes

import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import FlatParams, PlanFunction, PlanPool, precision_of
from .conv import Conv2d


def _l2normalize(v, eps=1e-12):
    """SpectralNorm.py:10-11"""
    return v / (v.norm() + eps)


class SpectralNorm(nn.Module):
    """Reference nets/SpectralNorm.py:14-68 (parameter holder).  The wrapped conv keeps the
    reference's parameters `weight_u`, `weight_v` (requires_grad False), `weight_bar` and
    `bias`, drawn in the reference's order, so state_dicts interchange.  `module.weight` is a
    non-persistent buffer (a plain attribute in the reference, so not in the state_dict) that
    receives W_bar / sigma from the owning discriminator's SpectralNorm launch before every
    forward; the conv kernels pack it like any other weight."""

    def __init__(self, module, name="weight", power_iterations=1):
        super().__init__()
        if name != "weight":
            raise NotImplementedError("SpectralNorm over a parameter other than `weight`")
        self.module, self.name, self.power_iterations = module, name, power_iterations
        w = module.weight
        height = w.data.shape[0]
        width = w.view(height, -1).data.shape[1]
        u = nn.Parameter(w.data.new(height).normal_(0, 1), requires_grad=False)
        v = nn.Parameter(w.data.new(width).normal_(0, 1), requires_grad=False)
        u.data = _l2normalize(u.data)
        v.data = _l2normalize(v.data)
        w_bar = nn.Parameter(w.data)
        del module._parameters[name]
        module.register_parameter(name + "_u", u)
        module.register_parameter(name + "_v", v)
        module.register_parameter(name + "_bar", w_bar)
        module.register_buffer(name, torch.zeros_like(w.data), persistent=False)
        self.h, self.width = height, width


def _conv_of(m):
    return m.module if isinstance(m, SpectralNorm) else m


class ResnetBlock(nn.Module):
    """conv - LeakyReLU(0.2) - conv, + input (no activation after the sum)."""

    def __init__(self, in_dim, out_dim, ks):
        super().__init__()
        self.conv = nn.Sequential(Conv2d(in_dim, out_dim, ks, stride=1, padding=ks // 2),
                                  nn.LeakyReLU(0.2, inplace=True),
                                  Conv2d(out_dim, out_dim, ks, stride=1, padding=ks // 2))


class ResnetSNBlock(nn.Module):
    """ResnetBlock with SpectralNorm convs (FrameDisc.py:21-32, VidDisc.py:21-32)."""

    def __init__(self, in_dim, out_dim, ks):
        super().__init__()
        self.conv = nn.Sequential(SpectralNorm(Conv2d(in_dim, out_dim, ks, stride=1, padding=ks // 2)),
                                  nn.LeakyReLU(0.2, inplace=True),
                                  SpectralNorm(Conv2d(out_dim, out_dim, ks, stride=1, padding=ks // 2)))


def _packing(widths):
    """Channel slices for the concatenated inputs: each input gets a 4-aligned slice, the
    last one stretched so the total is a multiple of 8 (every channel is written).
    -> (slices [(c0, c, ext_c)], cmap position -> concat channel or -1, total)"""
    slices, cmap, off, src = [], [], 0, 0
    for i, w in enumerate(widths):
        c = E.rup(w, 4)
        if i == len(widths) - 1:
            c = E.rup(off + c, E.PADC) - off
        slices.append((off, c, w))
        cmap += list(range(src, src + w)) + [-1] * (c - w)
        off += c
        src += w
    return slices, cmap, off


def lower_sequential(g, mods, x, prefix, trainable, cmap=None, out_key=None, head_c=None):
    """Lower an nn.Sequential of Conv2d / SpectralNorm(Conv2d) / ConvTranspose2d (each with
    an optional BatchNorm2d and LeakyReLU after it), ResnetBlock / ResnetSNBlock and a final
    AvgPool2d (head "score", head_c channels) into the engine graph `g`, starting from region
    `x`.  Buffers are named f"{prefix}.{i}" after the Sequential index (the activation names
    the oracles use).  A conv with nothing after it writes the external fp32 output
    `out_key`.  Returns the last region (None after an external output or a head)."""
    A = L
    i, first = 0, True
    while i < len(mods):
        m = mods[i]
        if isinstance(m, (nn.Conv2d, SpectralNorm, nn.ConvTranspose2d)):
            conv = _conv_of(m)
            tr = isinstance(conv, nn.ConvTranspose2d)
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            if tr:
                hh, ww = (x.H - 1) * s - 2 * p + k, (x.W - 1) * s - 2 * p + k
            else:
                hh, ww = (x.H + 2 * p - k) // s + 1, (x.W + 2 * p - k) // s + 1
            cm = cmap if first else None
            first = False
            name = f"{prefix}.{i}"

            def emit(src, dst, act, conv=conv, cm=cm, name=name, tr=tr):
                if tr:
                    assert cm is None, "a transposed conv cannot take a packed input map"
                    g.convT(src, conv, dst, act=act, trainable=trainable, name=name)
                else:
                    g.conv(src, conv, dst, act=act, cmap=cm, trainable=trainable, name=name)

            if nxt is None:  # the map is the output
                assert out_key is not None and not tr
                o = g.buffer(out_key, hh, ww, E.rup(conv.out_channels, 8), dtype=torch.float32, external=True)
                emit(x, E.R(o), A.ACT_NONE)
                g.output(out_key, E.R(o), conv.out_channels)
                return None
            if isinstance(nxt, nn.BatchNorm2d):
                act = A.ACT_LRELU if i + 2 < len(mods) and isinstance(mods[i + 2], nn.LeakyReLU) else A.ACT_NONE
                t = g.buffer(name, hh, ww, E.rup(conv.out_channels, 8))
                emit(x, E.R(t), A.ACT_NONE)
                o = g.buffer(f"{prefix}.{i + 1}", hh, ww, E.rup(conv.out_channels, 8))
                g.bn(E.R(t), nxt, E.R(o), act=act, trainable=trainable)
                x = E.R(o)
                i += 3 if act == A.ACT_LRELU else 2
                continue
            act = A.ACT_LRELU if isinstance(nxt, nn.LeakyReLU) else A.ACT_NONE
            o = g.buffer(name, hh, ww, E.rup(conv.out_channels, 8))
            emit(x, E.R(o), act)
            x = E.R(o)
            i += 2 if act == A.ACT_LRELU else 1
            continue
        if isinstance(m, (ResnetBlock, ResnetSNBlock)):
            c0, c2 = _conv_of(m.conv[0]), _conv_of(m.conv[2])
            h = g.buffer(f"{prefix}.{i}.h", x.H, x.W, E.rup(c0.out_channels, 8))
            g.conv(x, c0, E.R(h), act=A.ACT_LRELU, trainable=trainable, name=f"{prefix}.{i}.conv.0")
            o = g.buffer(f"{prefix}.{i}.out", x.H, x.W, E.rup(c2.out_channels, 8))
            g.conv(E.R(h), c2, E.R(o), res=x, trainable=trainable, name=f"{prefix}.{i}.conv.2")
            x = E.R(o)
            i += 1
            continue
        if isinstance(m, nn.AvgPool2d):
            k = m.kernel_size if isinstance(m.kernel_size, int) else m.kernel_size[0]
            assert head_c is not None and x.c == head_c
            g.head(x, k, "score")
            return None
        raise TypeError(f"unsupported layer {prefix}.{i}: {m}")
    return x


class _PlanDiscriminator(FlatParams, nn.Module):
    """Shared plan lowering / autograd plumbing of the discriminators."""

    in_keys = ()
    local = False  # True: the last conv's (B, 1, h, w) map is the output (no AvgPool head)
    plan_log = None  # test support: a list collects the plan of every forward call, in order

    def _finish_init(self):
        self.dtype = precision_of(self.args)
        self._pool = PlanPool(self._build_plan)
        self._sn = [m for m in self.modules() if isinstance(m, SpectralNorm)]
        self._flatten()

    def _in_widths(self):
        raise NotImplementedError

    def _lower(self, g, H, W, trainable, in_grads):
        A = L
        widths = self._in_widths()
        slices, cmap, total = _packing(widths)
        inp = g.buffer("disc_in", H, W, total)
        for k, (c0, c, w) in enumerate(slices):
            g.input_nchw(E.R(inp, c0, c), f"in{k}", ext_c=w, requires_grad=bool(in_grads[k]))
        assert self.local or self.out_c is not None
        lower_sequential(g, list(self.layer), E.R(inp), "layer", trainable, cmap=cmap,
                         out_key="score" if self.local else None, head_c=None if self.local else self.out_c)
        return g

    def _build_plan(self, key):
        n, H, W, dtype, bn_train, trainable, in_grads, backward, dev = key
        g = E.Graph(dtype)
        g.bn_training = bn_train
        self._lower(g, H, W, trainable, in_grads)
        return g.compile(n, dev, backward=backward)

    def _on_moved(self):
        self._pool.clear()

    # ---- SpectralNorm (nets/SpectralNorm.py:23-35 and its autograd) ----
    def _sn_state(self, plan, dev):
        sizes = [1 + s.h + s.width for s in self._sn]
        st = plan.__dict__.get("sn_state")
        if st is None:
            st = torch.zeros(sum(sizes), dtype=torch.float32, device=dev)
            plan.sn_state = st
        return st, sizes

    def _sn_forward(self, plan, dev):
        """power iteration of every SN layer (u, v updated in place; the values used saved in
        the plan's state for its backward) and W_bar / sigma into module.weight"""
        st, sizes = self._sn_state(plan, dev)
        arr = (L.SnLayer * len(self._sn))()
        off = 0
        for d, s, n in zip(arr, self._sn, sizes):
            m = s.module
            d.w_bar, d.u, d.v = m.weight_bar.data_ptr(), m.weight_u.data_ptr(), m.weight_v.data_ptr()
            d.w_eff = m.weight.data_ptr()
            d.state_off, d.h, d.width, d.power_iterations = off, s.h, s.width, s.power_iterations
            off += n
        L.check(L.load().dvie_sn_fwd(ctypes.addressof(arr), len(self._sn), st.data_ptr(), L.stream_ptr(dev)),
                "spectral norm forward")

    def _sn_backward(self, plan, accumulate, dev):
        """d(W_bar / sigma) (the plan's weight gradient of module.weight) -> weight_bar.grad,
        and u / v gradients once they are trainable (InterGANNet's set_net_grad(True))"""
        st, sizes = self._sn_state(plan, dev)
        todo, off = [], 0
        for s, n in zip(self._sn, sizes):
            m = s.module
            if m.weight_bar.grad is not None and m.weight.grad is not None:
                todo.append((s, off))
            off += n
        if not todo:
            return
        arr = (L.SnLayer * len(todo))()
        for d, (s, o) in zip(arr, todo):
            m = s.module
            d.w_bar, d.g_eff, d.g_bar = m.weight_bar.data_ptr(), m.weight.grad.data_ptr(), m.weight_bar.grad.data_ptr()
            d.g_u = m.weight_u.grad.data_ptr() if m.weight_u.grad is not None else None
            d.g_v = m.weight_v.grad.data_ptr() if m.weight_v.grad is not None else None
            d.state_off, d.h, d.width, d.beta = o, s.h, s.width, int(accumulate)
        L.check(L.load().dvie_sn_bwd(ctypes.addressof(arr), len(todo), st.data_ptr(), L.stream_ptr(dev)),
                "spectral norm backward")

    def run_forward(self, inputs, train):
        x = inputs[0]
        L.require_gpu(x)
        n, _, H, W = x.shape
        needs = getattr(self, "_in_needs", (False,) * len(inputs))
        trainable = bool(train) and any(p.requires_grad for p in self.parameters())
        in_grads = tuple(bool(train) and bool(k) for k in needs)
        backward = trainable or any(in_grads)
        key = (n, H, W, self.dtype, self.training, trainable, in_grads, backward, x.device)
        plan = self._pool.acquire(key)
        if self._sn:  # the reference updates u, v on every call, train or eval
            self._sn_forward(plan, x.device)
        for k, t in enumerate(inputs):
            plan.set_input(f"in{k}", t)
        if self.local:
            region, c = plan.g.outputs["score"]
            buf = torch.empty((n, region.H, region.W, region.buf.C), dtype=torch.float32, device=x.device)
            plan.set_output("score", buf)
            out = buf.permute(0, 3, 1, 2)[:, :c]
        else:
            hb = plan.g.heads["score"]
            rows = n * (hb.H // self.pool) * (hb.W // self.pool)
            out = torch.empty(rows, dtype=torch.float32, device=x.device)
            plan.set_head_output("score", out)
        plan.run_forward()
        self.last_plan = plan
        if self.plan_log is not None:
            self.plan_log.append(plan)
        if self.training:  # one increment per BatchNorm call, as nn.BatchNorm2d.train()
            for op in plan.g.ops:
                if isinstance(op, E.BNOp) and op.m.num_batches_tracked is not None:
                    op.m.num_batches_tracked.add_(1)
        return plan, (out,)

    def run_backward(self, plan, inputs, grads, needs):
        (go,) = grads
        dev = inputs[0].device
        pn = getattr(self, "_param_needs", None)
        sel = None if pn is None else [p for p, nd in zip(self._flat_params, pn) if nd]
        trainable = any(p.requires_grad for p in self.parameters()) if sel is None else bool(sel)
        accumulate = False
        if trainable:
            # (SpectralNorm u / v: a gradient only when they required one at the forward)
            accumulate = self.grad_views(sel)
            # SN convs: this call's d(W_bar / sigma) overwrites module.weight.grad (scratch)
            plan.set_param_grads(accumulate, fresh={id(s.module) for s in self._sn})
        if self.local:
            plan.set_output_grad("score", go.float())
        else:
            plan.set_head_grad("score", go.float())
        outs = []
        for k, t in enumerate(inputs):
            if f"in{k}" in plan.ext_grad:
                gx = torch.empty(t.shape, dtype=torch.float32, device=t.device)
                plan.set_input_grad(f"in{k}", gx)
                outs.append(gx)
            else:
                outs.append(None)
        plan.run_backward()
        if trainable and self._sn:
            self._sn_backward(plan, accumulate, dev)
        return outs

    def activation_signs(self):
        """branch taken by every LeakyReLU of the last forward (see Plan.activation_signs)"""
        return self.last_plan.activation_signs()

    def _run(self, *inputs):
        ins = [t.float() for t in inputs]
        params = [p for p in self._flat_params]
        return PlanFunction.apply(self, len(ins), *ins, *params)


class _FrameBase(_PlanDiscriminator):
    def _setup(self, args):
        self.args = args
        self.seg_disc = bool(getattr(args, "seg_disc", False))
        self.input_dim = 23 if self.seg_disc else 3

    def _in_widths(self):
        return [3, 20] if self.seg_disc else [3]

    def forward(self, x, seg=None, bboxes=None):
        return self._run(x, seg) if self.seg_disc else self._run(x)


class _VideoBase(_PlanDiscriminator):
    def _setup(self, args):
        self.args = args
        self.seg_disc = bool(getattr(args, "seg_disc", False))
        self.input_dim = 23 if self.seg_disc else 3

    def _in_widths(self):
        return [3, 20, 6, 40] if self.seg_disc else [3, 6]

    def forward(self, x, seg, input_x, input_seg, bboxes=None):
        if self.seg_disc:
            return self._run(x, seg, input_x, input_seg)
        return self._run(x, input_x)


def _lr(inplace=True):
    return nn.LeakyReLU(0.2, inplace=inplace)


def _sn(*a):
    return SpectralNorm(Conv2d(*a))


class FrameDiscriminator(_FrameBase):
    """Reference nets/FrameDisc.py:35-75."""

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            Conv2d(self.input_dim, 16, 3, 1, 1), _lr(False),
            Conv2d(16, 32, 5, 1, 2), nn.BatchNorm2d(32), _lr(False),
            Conv2d(32, 64, 3, 2, 1), _lr(), ResnetBlock(64, 64, 3),
            Conv2d(64, 96, 3, 2, 1), _lr(), ResnetBlock(96, 96, 3),
            Conv2d(96, 128, 3, 2, 1), _lr(), ResnetBlock(128, 128, 3),
            Conv2d(128, 192, 3, 2, 1), _lr(), ResnetBlock(192, 192, 3),
            Conv2d(192, 192, 3, 1, 1), nn.AvgPool2d(8))
        self.out_c, self.pool = 192, 8
        self._finish_init()


class FrameLocalDiscriminator(_FrameBase):
    """Reference nets/FrameDisc.py:77-114 (output: the (B, 1, H/4, W/4) map)."""
    local = True

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            Conv2d(self.input_dim, 16, 3, 1, 1), _lr(False),
            Conv2d(16, 32, 5, 1, 2), nn.BatchNorm2d(32), _lr(False),
            Conv2d(32, 64, 3, 2, 1), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 64, 3, 1, 1), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 128, 3, 2, 1), nn.BatchNorm2d(128), _lr(),
            Conv2d(128, 128, 3, 1, 1), nn.BatchNorm2d(128), _lr(),
            Conv2d(128, 64, 3, 1, 1), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 1, 1, 1, 0))
        self._finish_init()


class FrameSNDiscriminator(_FrameBase):
    """Reference nets/FrameDisc.py:116-156."""

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            _sn(self.input_dim, 16, 3, 1, 1), _lr(False),
            _sn(16, 32, 5, 1, 2), _lr(False),
            _sn(32, 64, 3, 2, 1), _lr(), ResnetSNBlock(64, 64, 3),
            _sn(64, 96, 3, 2, 1), _lr(), ResnetSNBlock(96, 96, 3),
            _sn(96, 128, 3, 2, 1), _lr(), ResnetSNBlock(128, 128, 3),
            _sn(128, 128, 3, 1, 1), nn.AvgPool2d(16))
        self.out_c, self.pool = 128, 16
        self._finish_init()


class FrameSNLocalDiscriminator(_FrameBase):
    """Reference nets/FrameDisc.py:158-189 (output: the (B, 1, H/4, W/4) map)."""
    local = True

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            _sn(self.input_dim, 16, 3, 1, 1), _lr(False),
            _sn(16, 32, 5, 1, 2), _lr(False),
            _sn(32, 64, 3, 2, 1), _lr(),
            _sn(64, 64, 3, 1, 1), _lr(),
            _sn(64, 128, 3, 2, 1), _lr(),
            _sn(128, 128, 3, 1, 1), _lr(),
            _sn(128, 64, 3, 1, 1), _lr(),
            _sn(64, 1, 1, 1, 0))
        self._finish_init()


class VideoDiscriminator(_VideoBase):
    """Reference nets/VidDisc.py:34-84."""

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            Conv2d(3 * self.input_dim, 32, 3, 1, 1), _lr(False),
            Conv2d(32, 64, 5, 1, 2), nn.BatchNorm2d(64), _lr(False),
            Conv2d(64, 32, 3, 1, 1), nn.BatchNorm2d(32), _lr(False),
            Conv2d(32, 32, 3, 2, 1), _lr(), ResnetBlock(32, 32, 3),
            Conv2d(32, 64, 3, 2, 1), _lr(), ResnetBlock(64, 64, 3),
            Conv2d(64, 128, 3, 2, 1), _lr(), ResnetBlock(128, 128, 3),
            Conv2d(128, 256, 3, 2, 1), _lr(), ResnetBlock(256, 256, 3),
            Conv2d(256, 256, 3, 1, 1), nn.AvgPool2d(8))
        self.out_c, self.pool = 256, 8
        self._finish_init()


class VideoLocalDiscriminator(_VideoBase):
    """Reference nets/VidDisc.py:86-138 (output: the (B, 1, H/16, W/16) map)."""
    local = True

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            Conv2d(3 * self.input_dim, 64, 1, 1, 0), _lr(False),
            Conv2d(64, 64, 3, 1, 1), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 64, 3, 2, 1), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 64, 3, 1, 1), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 64, 3, 1, 1), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 128, 3, 2, 1), nn.BatchNorm2d(128), _lr(),
            Conv2d(128, 128, 3, 1, 1), nn.BatchNorm2d(128), _lr(),
            Conv2d(128, 128, 3, 2, 1), nn.BatchNorm2d(128), _lr(),
            Conv2d(128, 128, 3, 1, 1), nn.BatchNorm2d(128), _lr(),
            Conv2d(128, 256, 3, 2, 1), nn.BatchNorm2d(256), _lr(),
            Conv2d(256, 256, 3, 1, 1), nn.BatchNorm2d(256), _lr(),
            Conv2d(256, 64, 1, 1, 0), nn.BatchNorm2d(64), _lr(),
            Conv2d(64, 1, 1, 1, 0))
        self._finish_init()


class VideoSNDiscriminator(_VideoBase):
    """Reference nets/VidDisc.py:140-183."""

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            _sn(3 * self.input_dim, 32, 3, 1, 1), _lr(False),
            _sn(32, 64, 5, 1, 2), _lr(False),
            _sn(64, 32, 3, 1, 1), _lr(False),
            _sn(32, 32, 3, 2, 1), _lr(), ResnetSNBlock(32, 32, 3),
            _sn(32, 64, 3, 2, 1), _lr(), ResnetSNBlock(64, 64, 3),
            _sn(64, 128, 3, 2, 1), _lr(), ResnetSNBlock(128, 128, 3),
            _sn(128, 128, 3, 1, 1), nn.AvgPool2d(16))
        self.out_c, self.pool = 128, 16
        self._finish_init()


class VideoSNLocalDiscriminator(_VideoBase):
    """Reference nets/VidDisc.py:185-226 (output: the (B, 1, H/16, W/16) map)."""
    local = True

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self.layer = nn.Sequential(
            _sn(3 * self.input_dim, 64, 1, 1, 0), _lr(False),
            _sn(64, 64, 3, 1, 1), _lr(),
            _sn(64, 64, 3, 2, 1), _lr(),
            _sn(64, 64, 3, 1, 1), _lr(),
            _sn(64, 64, 3, 1, 1), _lr(),
            _sn(64, 128, 3, 2, 1), _lr(),
            _sn(128, 128, 3, 1, 1), _lr(),
            _sn(128, 128, 3, 2, 1), _lr(),
            _sn(128, 128, 3, 1, 1), _lr(),
            _sn(128, 256, 3, 2, 1), _lr(),
            _sn(256, 256, 3, 1, 1), _lr(),
            _sn(256, 64, 1, 1, 0), _lr(),
            _sn(64, 1, 1, 1, 0))
        self._finish_init()
