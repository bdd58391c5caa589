"""Frame / video discriminators of InterGANNet on the MI355X plan engine.

Module trees, construction order (so seeded initialisation) and state_dict keys are those
of the reference: FrameDiscriminator nets/FrameDisc.py:35-75, VideoDiscriminator
nets/VidDisc.py:34-84, ResnetBlock FrameDisc.py:8-19 / VidDisc.py:8-19.  The forward and
backward do not run the submodules: `_lower` turns `self.layer` into one engine plan
(HIP convs with fused bias / residual / LeakyReLU epilogues, BatchNorm with batch
statistics fused with its LeakyReLU, and the AvgPool + view(-1, C).mean(1) head).

Calling conventions follow the reference: FrameDiscriminator(x, seg, bboxes=None) and
VideoDiscriminator(x, seg, input_x, input_seg, bboxes=None) -> (B*k,) scores, where k is
the number of pooled cells (k = 1 at the reference's 128x128 training crops).  The input
concat (`torch.cat` in the reference forward) is never materialised: each input is packed
into its own channel slice of the first conv's input buffer.
"""
import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import FlatParams, PlanFunction, PlanPool, precision_of
from .conv import Conv2d


class ResnetBlock(nn.Module):
    """conv - LeakyReLU(0.2) - conv, + input (no activation after the sum)."""

    def __init__(self, in_dim, out_dim, ks):
        super().__init__()
        self.conv = nn.Sequential(Conv2d(in_dim, out_dim, ks, stride=1, padding=ks // 2),
                                  nn.LeakyReLU(0.2, inplace=True),
                                  Conv2d(out_dim, out_dim, ks, stride=1, padding=ks // 2))


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


class _PlanDiscriminator(FlatParams, nn.Module):
    """Shared plan lowering / autograd plumbing of the two discriminators."""

    in_keys = ()

    def _finish_init(self):
        self.dtype = precision_of(self.args)
        self._pool = PlanPool(self._build_plan)
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
        x = E.R(inp)
        mods = list(self.layer)
        i, first = 0, True
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.Conv2d):
                nxt = mods[i + 1] if i + 1 < len(mods) else None
                hh = (x.H + 2 * m.padding[0] - m.kernel_size[0]) // m.stride[0] + 1
                ww = (x.W + 2 * m.padding[1] - m.kernel_size[1]) // m.stride[1] + 1
                cm = cmap if first else None
                first = False
                if isinstance(nxt, nn.BatchNorm2d):
                    act = A.ACT_LRELU if i + 2 < len(mods) and isinstance(mods[i + 2], nn.LeakyReLU) else A.ACT_NONE
                    t = g.buffer(f"layer.{i}", hh, ww, E.rup(m.out_channels, 8))
                    g.conv(x, m, E.R(t), cmap=cm, trainable=trainable, name=f"layer.{i}")
                    o = g.buffer(f"layer.{i + 1}", hh, ww, E.rup(m.out_channels, 8))
                    g.bn(E.R(t), nxt, E.R(o), act=act, trainable=trainable)
                    x = E.R(o)
                    i += 3 if act == A.ACT_LRELU else 2
                    continue
                act = A.ACT_LRELU if isinstance(nxt, nn.LeakyReLU) else A.ACT_NONE
                o = g.buffer(f"layer.{i}", hh, ww, E.rup(m.out_channels, 8))
                g.conv(x, m, E.R(o), act=act, cmap=cm, trainable=trainable, name=f"layer.{i}")
                x = E.R(o)
                i += 2 if act == A.ACT_LRELU else 1
                continue
            if isinstance(m, ResnetBlock):
                c0, c2 = m.conv[0], m.conv[2]
                h = g.buffer(f"layer.{i}.h", x.H, x.W, E.rup(c0.out_channels, 8))
                g.conv(x, c0, E.R(h), act=A.ACT_LRELU, trainable=trainable, name=f"layer.{i}.conv.0")
                o = g.buffer(f"layer.{i}.out", x.H, x.W, E.rup(c2.out_channels, 8))
                g.conv(E.R(h), c2, E.R(o), res=x, trainable=trainable, name=f"layer.{i}.conv.2")
                x = E.R(o)
                i += 1
                continue
            if isinstance(m, nn.AvgPool2d):
                k = m.kernel_size if isinstance(m.kernel_size, int) else m.kernel_size[0]
                assert x.c == self.out_c
                g.head(x, k, "score")
                i += 1
                continue
            raise TypeError(f"unsupported discriminator layer {i}: {m}")
        return g

    def _build_plan(self, key):
        n, H, W, dtype, bn_train, trainable, in_grads, backward, dev = key
        g = E.Graph(dtype)
        g.bn_training = bn_train
        self._lower(g, H, W, trainable, in_grads)
        return g.compile(n, dev, backward=backward)

    def _on_moved(self):
        self._pool.clear()

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
        for k, t in enumerate(inputs):
            plan.set_input(f"in{k}", t)
        hb = plan.g.heads["score"]
        rows = n * (hb.H // self.pool) * (hb.W // self.pool)
        out = torch.empty(rows, dtype=torch.float32, device=x.device)
        plan.set_head_output("score", out)
        plan.run_forward()
        self.last_plan = plan
        if self.training:  # one increment per BatchNorm call, as nn.BatchNorm2d.train()
            for op in plan.g.ops:
                if isinstance(op, E.BNOp) and op.m.num_batches_tracked is not None:
                    op.m.num_batches_tracked.add_(1)
        return plan, (out,)

    def run_backward(self, plan, inputs, grads, needs):
        (go,) = grads
        if any(p.requires_grad for p in self.parameters()):
            plan.set_param_grads(self.grad_views())
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
        return outs

    def activation_signs(self):
        """branch taken by every LeakyReLU of the last forward (see Plan.activation_signs)"""
        return self.last_plan.activation_signs()

    def _run(self, *inputs):
        ins = [t.float() for t in inputs]
        params = [p for p in self._flat_params]
        return PlanFunction.apply(self, len(ins), *ins, *params)


class FrameDiscriminator(_PlanDiscriminator):
    """Reference nets/FrameDisc.py:35-75."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.seg_disc = bool(getattr(args, "seg_disc", False))
        self.input_dim = 23 if self.seg_disc else 3
        self.layer = nn.Sequential(
            Conv2d(self.input_dim, 16, 3, 1, 1), nn.LeakyReLU(0.2, inplace=False),
            Conv2d(16, 32, 5, 1, 2), nn.BatchNorm2d(32), nn.LeakyReLU(0.2, inplace=False),
            Conv2d(32, 64, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(64, 64, 3),
            Conv2d(64, 96, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(96, 96, 3),
            Conv2d(96, 128, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(128, 128, 3),
            Conv2d(128, 192, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(192, 192, 3),
            Conv2d(192, 192, 3, 1, 1), nn.AvgPool2d(8))
        self.out_c, self.pool = 192, 8
        self._finish_init()

    def _in_widths(self):
        return [3, 20] if self.seg_disc else [3]

    def forward(self, x, seg=None, bboxes=None):
        return self._run(x, seg) if self.seg_disc else self._run(x)


class VideoDiscriminator(_PlanDiscriminator):
    """Reference nets/VidDisc.py:34-84."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.seg_disc = bool(getattr(args, "seg_disc", False))
        self.input_dim = 23 if self.seg_disc else 3
        self.layer = nn.Sequential(
            Conv2d(3 * self.input_dim, 32, 3, 1, 1), nn.LeakyReLU(0.2, inplace=False),
            Conv2d(32, 64, 5, 1, 2), nn.BatchNorm2d(64), nn.LeakyReLU(0.2, inplace=False),
            Conv2d(64, 32, 3, 1, 1), nn.BatchNorm2d(32), nn.LeakyReLU(0.2, inplace=False),
            Conv2d(32, 32, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(32, 32, 3),
            Conv2d(32, 64, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(64, 64, 3),
            Conv2d(64, 128, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(128, 128, 3),
            Conv2d(128, 256, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), ResnetBlock(256, 256, 3),
            Conv2d(256, 256, 3, 1, 1), nn.AvgPool2d(8))
        self.out_c, self.pool = 256, 8
        self._finish_init()

    def _in_widths(self):
        return [3, 20, 6, 40] if self.seg_disc else [3, 6]

    def forward(self, x, seg, input_x, input_seg, bboxes=None):
        if self.seg_disc:
            return self._run(x, seg, input_x, input_seg)
        return self._run(x, input_x)
