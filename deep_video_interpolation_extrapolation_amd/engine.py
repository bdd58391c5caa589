"""Plan compiler for the MI355X frame-synthesis path.

A network (HRNet coarse generator, VGG19 perceptual features, ...) is described once with
a small builder API (`Graph.conv / fuse / pool / input_nchw / l1feat`).  `Graph.compile`
turns it into two flat descriptor lists for the C ABI (include/dvie.h):

* forward:  weight packing (one launch for all layers) + one descriptor per op;
* backward: derived here by reverse traversal.  Gradient contributions to a buffer are
  collected and emitted only when the last one is known, so that
  - the first contribution overwrites and the rest accumulate (epilogue `beta`),
  - identity contributions (residual adds, same-resolution fuse terms) ride along as the
    `res` operand of a kernel contribution instead of costing a pass of their own,
  - the producer's activation derivative (LeakyReLU/ELU/ReLU, computed from its output)
    is applied by the epilogue of the last contribution, so every buffer's gradient is
    already the pre-activation gradient the producer's wgrad/dgrad need.

Each list runs with a single host call (`dvie_run_ops`) on the current HIP stream.
All activations are NHWC buffers allocated once per (batch, height, width) plan; the
kernels never allocate.  Reference semantics: nets/HRNet.py, nets/vgg.py, losses.py.
"""
import ctypes
import math
import os

import torch

from . import _lib as L

PADC = 8  # channel padding granule (16-byte bf16 vectors)
PROFILE = None  # set to a list to time every op with HIP events (bench profiling steps)
DEBUG_NAN = bool(os.environ.get("DVIE_DEBUG_NAN"))  # op-by-op non-finite tracing (diagnostics only)
# DVIE_WGRAD_LANE=0: weight gradients on the caller's stream with everything else (A/B runs;
# read when a plan is compiled)
def _wgrad_lane():
    return os.environ.get("DVIE_WGRAD_LANE", "1") != "0"


# test support: hook(plan, arr, i, meta, run) is handed every executed op and calls run() to
# launch it (layer-local parity checks, tests/test_gpu_layers.py); None in the product
OP_HOOK = None


def pack_blocks(d):
    """workgroups dvie_pack_weights gives descriptor d (the library's own count: its block
    kinds are a function of the descriptor, csrc/conv.hip pack_kind)"""
    n = L.load().dvie_pack_blocks(ctypes.byref(d))
    assert n > 0, "dvie_pack_blocks: empty pack descriptor"
    return n


def _reduce_meta(name, r):
    """profiling meta of a slab reduction: the partial slabs read once, the gradient
    written (and read when accumulating)."""
    rows = r.ws_rows - r.co_off
    out = r.cout_p * r.cin_p * r.kh_n * r.kw_n
    return dict(cls="wgrad_reduce", name=name, flops=0.0,
                bytes=float(4 * (r.splits * rows * r.ws_k + out * (1 + r.beta))))


def rup(x, m):
    return (x + m - 1) // m * m


def elem_size(dt):
    return 2 if dt == torch.bfloat16 else 4


def dv_dtype(dt):
    return L.BF16 if dt == torch.bfloat16 else L.F32


class Buffer:
    """NHWC activation buffer [N, H, W, C] (C is also the pixel stride)."""

    def __init__(self, name, H, W, C, dtype=None, external=False):
        self.name, self.H, self.W, self.C = name, H, W, C
        self.dtype = dtype  # None -> graph compute dtype
        self.external = external
        self.t = None  # forward storage
        self.g = None  # gradient storage [Nb, H, W, C] (compute dtype)
        self.needs_grad = False
        self.producers = []
        self.consumers = []  # (op, region)
        self.expected = {}  # read region key -> number of gradient contributions
        self.pending = {}  # read region key -> contributions recorded so far

    def __repr__(self):
        return f"Buffer({self.name},{self.H}x{self.W}x{self.C})"


class Region:
    """Channel slice [c0, c0 + c) of a buffer."""

    def __init__(self, buf, c0=0, c=None):
        self.buf, self.c0 = buf, c0
        self.c = buf.C - c0 if c is None else c
        assert 0 <= c0 and c0 + self.c <= buf.C, (buf, c0, c)

    def key(self):
        return (self.c0, self.c)

    @property
    def H(self):
        return self.buf.H

    @property
    def W(self):
        return self.buf.W


def R(buf, c0=0, c=None):
    return Region(buf, c0, c)


class ConvLayer:
    """Packing/gradient metadata for one nn.Conv2d-shaped parameter set (OIHW fp32)."""

    def __init__(self, module, trainable=True, name=""):
        self.m = module
        self.name = name
        w = module.weight
        # nn.ConvTranspose2d: its (in, out, kh, kw) weight IS the OIHW weight of the conv
        # out -> in whose data gradient the transposed conv computes ("virtual conv": cout =
        # the ConvT input channels, cin = its output channels; the bias has cin entries)
        self.transposed = isinstance(module, torch.nn.ConvTranspose2d)
        if self.transposed:
            assert tuple(module.output_padding) == (0, 0), "ConvTranspose2d output_padding"
        if w.dim() == 2:  # nn.Linear (through LinearAsConv): a 1x1 conv over a (B, 1, 1, in) image
            self.cout, self.cin = w.shape
            self.kh = self.kw = 1
        else:
            self.cout, self.cin, self.kh, self.kw = w.shape
        self.stride = module.stride[0]
        self.pad = module.padding[0]
        assert module.stride[0] == module.stride[1] and module.padding[0] == module.padding[1]
        dil = tuple(getattr(module, "dilation", (1, 1)))
        assert dil[0] == dil[1] and module.groups == 1
        self.dil = dil[0]  # atrous convs (nets/refine_nets.py:60-69,210-219): taps dil apart
        assert self.dil == 1 or (self.stride == 1 and not isinstance(module, torch.nn.ConvTranspose2d)), \
            "dilation > 1 needs stride 1"
        self.has_bias = module.bias is not None
        self.trainable = trainable
        self.cmap = None  # packed input position -> source input channel (or -1)
        self.cin_p = None  # packed input channels
        self.cout_p = rup(self.cout, PADC)
        self.wf = None  # packed forward weights
        self.wd = []  # per dgrad phase: (tensor, taps(dict))
        self.bias_p = None
        self.uses = 0

    def bind_input(self, cin_p, cmap):
        if cmap is None:
            cmap = list(range(self.cin)) + [-1] * (cin_p - self.cin)
        assert len(cmap) == cin_p and cin_p >= self.cin
        if self.cin_p is None:
            self.cin_p, self.cmap = cin_p, list(cmap)
        else:
            assert self.cin_p == cin_p and self.cmap == list(cmap), f"{self.name}: inconsistent input packing"

    def fwd_taps(self):
        d = self.dil
        return dict(th=self.kh, tw=self.kw, dy0=-self.pad, dx0=-self.pad, ddy=d, ddx=d, kh0=0, kw0=0, dkh=1, dkw=1)

    def dgrad_phases(self, H, W):
        """Stride-s data gradient as s*s stride-1 convs over the output gradient."""
        s, p = self.stride, self.pad
        if s == 1:  # one phase; taps by increasing input offset p - k*dil, k = kh-1 .. 0
            d = self.dil
            return [dict(ry=0, rx=0, oh=H, ow=W, th=self.kh, tw=self.kw, kh0=self.kh - 1, kw0=self.kw - 1,
                         dkh=-1, dkw=-1, dy0=p - (self.kh - 1) * d, dx0=p - (self.kw - 1) * d, ddy=d, ddx=d)]
        phases = []
        for ry in range(s):
            khs = [k for k in range(self.kh) if (ry + p - k) % s == 0]
            if not khs:
                continue
            for rx in range(s):
                kws = [k for k in range(self.kw) if (rx + p - k) % s == 0]
                if not kws:
                    continue
                oh = (H - ry + s - 1) // s
                ow = (W - rx + s - 1) // s
                if oh <= 0 or ow <= 0:
                    continue
                # taps ordered by increasing input offset (ddy = ddx = +1): tap i reads
                # dy0 + i and weight row khs[-1] - i*s
                th, tw = len(khs), len(kws)
                phases.append(dict(ry=ry, rx=rx, oh=oh, ow=ow, th=th, tw=tw, kh0=khs[-1], kw0=kws[-1],
                                   dkh=-s, dkw=-s, dy0=(ry + p - khs[0]) // s - (th - 1),
                                   dx0=(rx + p - kws[0]) // s - (tw - 1), ddy=1, ddx=1))
        return phases


class _Op:
    pass


class ConvOp(_Op):
    def __init__(self, x, layer, out, act, res):
        self.x, self.layer, self.out, self.act, self.res = x, layer, out, act, res

    def inputs(self):
        return [self.x] + ([self.res] if self.res is not None else [])


class ConvTOp(_Op):
    """nn.ConvTranspose2d (+ activation): x (ConvT input) -> out (ConvT output)."""

    def __init__(self, x, layer, out, act):
        self.x, self.layer, self.out, self.act, self.res = x, layer, out, act, None

    def inputs(self):
        return [self.x]


class LinearAsConv:
    """nn.Linear seen by the engine as a 1x1 conv (the same (out, in) weight memory)."""
    stride, padding, dilation, groups = (1, 1), (0, 0), (1, 1), 1

    def __init__(self, linear):
        self.lin = linear

    @property
    def weight(self):
        return self.lin.weight

    @property
    def bias(self):
        return self.lin.bias


class StackedConv:
    """Several convs of one input run as ONE conv whose output channels are the parts'
    outputs stacked in order (e.g. HRNet's rgb_layer.0 / seg_layer.0, both 1x1 448 -> 448
    over the same concat: one 448 -> 896 GEMM reads the concat once, and its data gradient
    sums both heads' contributions in one K = 896 reduction).  The parts' weights must be
    consecutive in memory, and so must their biases and their .grad views (FlatParams lays
    the parameters out in `params()` order); `contiguous()` checks it."""

    def __init__(self, parts):
        self.parts = list(parts)
        m0 = self.parts[0]
        self.stride, self.padding = m0.stride, m0.padding
        self.dilation, self.groups = getattr(m0, "dilation", (1, 1)), m0.groups
        for m in self.parts:
            assert (m.stride, m.padding, m.groups, tuple(m.weight.shape[1:])) == \
                (m0.stride, m0.padding, m0.groups, tuple(m0.weight.shape[1:]))
            assert (m.bias is None) == (m0.bias is None)

    def params(self):
        """flat-buffer order: all weights, then all biases"""
        return [m.weight for m in self.parts] + [m.bias for m in self.parts if m.bias is not None]

    @staticmethod
    def _stack(ts):
        t0 = ts[0]
        shape = (sum(t.shape[0] for t in ts),) + tuple(t0.shape[1:])
        return torch.as_strided(t0, shape, t0.stride(), t0.storage_offset())

    @staticmethod
    def _consecutive(ts):
        return all(b.data_ptr() == a.data_ptr() + a.numel() * a.element_size() and a.is_contiguous() and b.is_contiguous()
                   and a.dtype == b.dtype for a, b in zip(ts, ts[1:]))

    def contiguous(self, grads=False):
        ws = [m.weight for m in self.parts]
        bs = [m.bias for m in self.parts if m.bias is not None]
        ok = self._consecutive(ws) and (not bs or self._consecutive(bs))
        if grads:
            ok = ok and all(t.grad is not None for t in ws + bs) and self._consecutive([t.grad for t in ws]) and (
                not bs or self._consecutive([t.grad for t in bs]))
        return ok

    def _view(self, ts):
        # not (yet) consecutive, e.g. the shape-only lowering before FlatParams lays the
        # parameters out: a meta tensor of the stacked shape (packing asserts contiguity)
        if self._consecutive(ts):
            return self._stack(ts)
        return torch.empty((sum(t.shape[0] for t in ts),) + tuple(ts[0].shape[1:]), device="meta")

    @property
    def weight(self):
        return self._view([m.weight for m in self.parts])

    @property
    def bias(self):
        if self.parts[0].bias is None:
            return None
        return self._view([m.bias for m in self.parts])

    def grad_ptr(self, which):
        """device pointer of the stacked gradient of `which` (the first part's .grad)"""
        ts = [getattr(m, which) for m in self.parts]
        for t in ts:
            if t.grad is None:
                t.grad = torch.zeros_like(t)
        assert self._consecutive([t.grad for t in ts]), "StackedConv: part gradients are not consecutive"
        return ts[0].grad.data_ptr()


class FuseOp(_Op):
    """out = act(sum of the srcs, each bilinearly resized to out's grid).  detach: no
    gradient flows back to the srcs (the reference's .detach() before an interpolate,
    e.g. nets/refine_nets.py:111)."""

    def __init__(self, srcs, out, act, align=False, detach=False):
        self.srcs, self.out, self.act, self.align, self.detach = srcs, out, act, align, detach

    def inputs(self):
        return list(self.srcs)


class AttnOp(_Op):
    """One dvie_attn op (kind: l2norm / corr / softmax / wnorm / gather / pool) reading `a`
    and the target maps `bs`, writing `out`; c = the channels it reduces or writes."""

    def __init__(self, kind, a, bs, out, c, wh=1, ww=1, nhalf=1, half0=0):
        self.kind, self.a, self.bs, self.out, self.c = kind, a, list(bs), out, c
        self.wh, self.ww, self.nhalf, self.half0 = wh, ww, nhalf, half0
        self.act = L.ACT_NONE

    def inputs(self):
        return [self.a] + self.bs


class PoolOp(_Op):
    def __init__(self, x, out):
        self.x, self.out, self.act = x, out, L.ACT_NONE

    def inputs(self):
        return [self.x]


class InputOp(_Op):
    """NCHW fp32 external tensor -> NHWC region.  `part` None: the whole batch;
    0 / 1: first / second half of the plan batch (VGG runs [pred | target])."""

    def __init__(self, out, key, part, ext_c0, ext_c, normalize, requires_grad):
        self.out, self.key, self.part, self.ext_c0, self.ext_c = out, key, part, ext_c0, ext_c
        self.normalize, self.requires_grad, self.act = normalize, requires_grad, L.ACT_NONE

    def inputs(self):
        return []


class L1FeatOp(_Op):
    """mean |f(pred) - f(gt)| of a feature buffer holding [pred batch | gt batch]."""

    def __init__(self, a, idx, weight):
        self.a, self.idx, self.weight, self.out, self.act = a, idx, weight, None, L.ACT_NONE

    def inputs(self):
        return [self.a]


class BNOp(_Op):
    """BatchNorm2d (+ activation) of a conv output buffer (reference nn.BatchNorm2d in
    nets/FrameDisc.py / nets/VidDisc.py / VAEHRNet).  x must be read by this op only."""

    def __init__(self, x, module, out, act, trainable):
        self.x, self.m, self.out, self.act, self.trainable = x, module, out, act, trainable

    def inputs(self):
        return [self.x]


class MaskOp(_Op):
    """out = src * m (or src * (1 - m)), m = channel `chan` of an external NCHW fp32 mask
    (the fg/bg split of nets/SepUNet.py:45-46).  The mask is data: no gradient to it."""

    def __init__(self, src, out, key, chan, inverse):
        self.src, self.out, self.key, self.chan, self.inverse, self.act = src, out, key, chan, inverse, L.ACT_NONE

    def inputs(self):
        return [self.src]


class OutNCHWOp(_Op):
    """Sink: copy an internal region to an external NCHW fp32 tensor (outputs whose
    producer carries an activation, e.g. the tanh RGB head of UNet/SepUNet)."""

    def __init__(self, region, key, channels):
        self.region, self.key, self.channels, self.out, self.act = region, key, channels, None, L.ACT_NONE

    def inputs(self):
        return []


class HeadOp(_Op):
    """AvgPool2d(pool) + view(-1, C).mean(1) -> external fp32 vector `key`."""

    def __init__(self, x, pool, key):
        self.x, self.pool, self.key, self.out, self.act = x, pool, key, None, L.ACT_NONE

    def inputs(self):
        return [self.x]


_IMAGENET_MEAN = [0.485, 0.456, 0.406]
_IMAGENET_STD = [0.229, 0.224, 0.225]


class Graph:
    def __init__(self, dtype=torch.float32):
        self.dtype = dtype
        self.ops = []
        self.buffers = []
        self.layers = []
        self.outputs = {}
        self.n_l1 = 0

    # ---------------- builder ----------------
    def buffer(self, name, H, W, C, dtype=None, external=False):
        b = Buffer(name, H, W, C, dtype, external)
        self.buffers.append(b)
        return b

    def layer(self, module, trainable=True, name=""):
        for lay in self.layers:
            if lay.m is module:
                return lay
        lay = ConvLayer(module, trainable, name)
        self.layers.append(lay)
        return lay

    def input_nchw(self, out, key, part=None, ext_c0=0, ext_c=None, normalize=False, requires_grad=False):
        assert not (requires_grad and part == 1)
        op = InputOp(out, key, part, ext_c0, out.c if ext_c is None else ext_c, normalize, requires_grad)
        self._add(op)
        return out

    def conv(self, x, module, out, act=L.ACT_NONE, res=None, cmap=None, trainable=True, name=""):
        lay = self.layer(module, trainable, name)
        lay.bind_input(x.c, cmap)
        assert out.c == lay.cout_p, (name, out.c, lay.cout_p)
        oh = (x.H + 2 * lay.pad - lay.dil * (lay.kh - 1) - 1) // lay.stride + 1
        ow = (x.W + 2 * lay.pad - lay.dil * (lay.kw - 1) - 1) // lay.stride + 1
        assert (out.H, out.W) == (oh, ow), (name, out.H, out.W, oh, ow)
        if res is not None:
            assert (res.H, res.W, res.c) == (out.H, out.W, out.c)
        self._add(ConvOp(x, lay, out, act, res))
        return out

    def convT(self, x, module, out, act=L.ACT_NONE, trainable=True, name=""):
        """nn.ConvTranspose2d: the data gradient of the conv sharing its weight
        (Conv2d(out_T -> in_T, k, s, p)), run as a forward op; out = (x - 1)*s - 2p + k."""
        lay = self.layer(module, trainable, name)
        assert lay.transposed
        lay.bind_input(out.c, None)
        assert x.c == lay.cout_p, (name, x.c, lay.cout_p)
        oh = (out.H + 2 * lay.pad - lay.kh) // lay.stride + 1
        ow = (out.W + 2 * lay.pad - lay.kw) // lay.stride + 1
        assert (x.H, x.W) == (oh, ow), (name, x.H, x.W, oh, ow)
        self._add(ConvTOp(x, lay, out, act))
        return out

    def fuse(self, srcs, out, act=L.ACT_NONE, align=False, detach=False):
        assert 1 <= len(srcs) <= 3
        for s in srcs:
            assert s.c == out.c
        self._add(FuseOp(srcs, out, act, align, detach))
        return out

    # ---- local-window attention (dvie_attn; MSResAttnRefine, nets/refine_nets.py:253-323) ----
    def l2norm(self, x, out):
        """out = x / |x| over the channels of each pixel."""
        assert (x.H, x.W, x.c) == (out.H, out.W, out.c)
        self._add(AttnOp("l2norm", x, [], out, x.c))
        return out

    def corr(self, x, targets, out, wh, ww):
        """out[p, m*K + k] = <x(p), targets[m](p + o_k)> (K = wh*ww window entries)."""
        K = wh * ww
        assert out.c >= len(targets) * K and all(t.c == x.c and (t.H, t.W) == (x.H, x.W) for t in targets)
        self._add(AttnOp("corr", x, list(targets), out, x.c, wh=wh, ww=ww, nhalf=len(targets)))
        return out

    def softmax(self, x, out, nhalf, wh, ww):
        """softmax over the first nhalf*wh*ww channels of each pixel."""
        self._add(AttnOp("softmax", x, [], out, x.c, wh=wh, ww=ww, nhalf=nhalf))
        return out

    def wnorm(self, x, out, nhalf, wh, ww):
        """per map m: out[:, m*K:(m+1)*K] = x / sum over those K channels."""
        self._add(AttnOp("wnorm", x, [], out, x.c, wh=wh, ww=ww, nhalf=nhalf))
        return out

    def gather(self, w, feats, out, half0, nhalf, wh, ww):
        """out(p) = sum_m sum_k w[p, (half0+m)*K + k] * feats[m](p + o_k)."""
        assert all(f.c == out.c and (f.H, f.W) == (out.H, out.W) for f in feats) and 1 <= len(feats) <= 2
        self._add(AttnOp("gather", w, list(feats), out, out.c, wh=wh, ww=ww, nhalf=nhalf, half0=half0))
        return out

    def apool(self, x, out, ph, pw):
        """F.avg_pool2d(x, (ph, pw), stride 1, padding (ph//2, pw//2), count_include_pad=False)."""
        assert (x.H, x.W, x.c) == (out.H, out.W, out.c)
        self._add(AttnOp("pool", x, [], out, x.c, wh=ph, ww=pw))
        return out

    def mask(self, src, out, key, chan, inverse=False):
        assert (src.H, src.W, src.c) == (out.H, out.W, out.c)
        self._add(MaskOp(src, out, key, chan, inverse))
        return out

    def output_nchw(self, key, region, channels):
        self._add(OutNCHWOp(region, key, channels))
        self.outputs[key] = (region, channels)

    def export_nchw(self, key, region, channels):
        """Copy a region to an external NCHW fp32 tensor with no gradient path (a detached
        side output, e.g. HRNet's seg-encoder features for the refinement stage)."""
        self._add(OutNCHWOp(region, key, channels))

    def pool(self, x, out):
        assert (out.H * 2, out.W * 2, out.c) == (x.H, x.W, x.c)
        self._add(PoolOp(x, out))
        return out

    def bn(self, x, module, out, act=L.ACT_NONE, trainable=True):
        """x: a conv output buffer read only by this op; it is kept in fp32 whatever the
        compute dtype (x - mean loses 2^-9 * |mean| / std relative precision in bf16)."""
        assert (x.H, x.W, x.c) == (out.H, out.W, out.c) and x.c == rup(module.num_features, PADC)
        x.buf.dtype = torch.float32
        self._add(BNOp(x, module, out, act, trainable))
        return out

    def head(self, x, pool, key):
        assert x.H >= pool and x.W >= pool
        self._add(HeadOp(x, pool, key))
        self.heads = getattr(self, "heads", {})
        self.heads[key] = x
        return key

    def l1feat(self, a, weight=1.0):
        op = L1FeatOp(a, self.n_l1, weight)
        self.n_l1 += 1
        self._add(op)
        return op.idx

    def output(self, key, region, channels):
        self.outputs[key] = (region, channels)

    def segenc_chain(self, ops):
        """mark three ConvOps as HRNet's segmentation encoder (conv + ELU, conv + ELU, conv):
        the plan runs their forward as one dvie_segenc_fwd launch where the shapes allow
        (Plan._segenc_fwd); their backward is unchanged."""
        self.__dict__.setdefault("segenc", []).append(tuple(ops))

    def _add(self, op):
        self.ops.append(op)
        if op.out is not None:
            op.out.buf.producers.append(op)
        for r in op.inputs():
            r.buf.consumers.append((op, r))

    # ---------------- compile ----------------
    def compile(self, n_fwd, device, n_bwd=None, backward=True):
        return Plan(self, n_fwd, n_fwd if n_bwd is None else n_bwd, device, backward)


class Plan:
    """Allocated buffers + forward/backward descriptor lists of one graph and shape."""

    def __init__(self, g, nf, nb, device, backward):
        self.g, self.nf, self.nb, self.device = g, nf, nb, device
        self.dtype = g.dtype
        self.dt = dv_dtype(g.dtype)
        self.es = elem_size(g.dtype)
        self.vec = 16 // self.es
        self.backward_enabled = backward
        self.keep = []  # tensors referenced by raw pointers
        self.busy = False
        self.generation = 0
        self.static_weights = False  # set by owners whose weights never train (nets/vgg.py)
        self._pack_srcs, self._pack_sig = [], None
        self._alloc()
        self.fwd = []
        self.bwd = []
        self._l1_fwd = []  # (forward list index, level) of the VGG feature-L1 loss ops
        self.ext_in = {}  # key -> list of (op index, InputOp) for patching
        self.ext_out = {}
        self.ext_grad = {}  # key -> list of bwd op indices (TONCHW)
        self._grad_slots = []  # (bwd index, layer, 'weight'|'bias', first use)
        self.ext_ograd = {}  # output key -> bwd op index of its gradient pack
        self.ws_floats = 1
        self._build_pack()
        self._build_forward()
        if backward:
            self._build_backward()
        self._finalize()

    # ---------------- allocation ----------------
    def _alloc(self):
        g = self.g
        for b in g.buffers:
            dt = b.dtype or self.dtype
            b.dt = dt
            if b.external:
                b.t = None
            else:
                b.t = torch.empty((self.nf, b.H, b.W, b.C), dtype=dt, device=self.device)
        # gradient requirements
        if self.backward_enabled:
            for op in g.ops:
                if op.out is None:
                    continue
                need = False
                if isinstance(op, InputOp):
                    need = op.requires_grad
                elif isinstance(op, (ConvOp, ConvTOp)):
                    need = op.layer.trainable or any(r.buf.needs_grad for r in op.inputs())
                elif isinstance(op, BNOp):
                    need = op.trainable or op.x.buf.needs_grad
                elif isinstance(op, FuseOp) and op.detach:
                    need = False
                else:
                    need = any(r.buf.needs_grad for r in op.inputs())
                op.out.buf.needs_grad = op.out.buf.needs_grad or need
            # the hidden maps of a segmentation encoder whose backward is one dvie_segenc_bwd
            # launch get no gradient storage: d_e1 / d_e2 stay on chip in that kernel
            self._seg_bwd = self._segenc_bwd_chains()
            self._seg_inner = {id(op.out.buf) for ch in self._seg_bwd.values() for op in ch[:2]}
            for b in g.buffers:
                if b.needs_grad and id(b) not in self._seg_inner:
                    b.g = torch.zeros((self.nb, b.H, b.W, b.C), dtype=self.dtype, device=self.device)
            for b in g.buffers:
                b.expected = {}
                b.pending = {}
                b.n_flushed = 0
                b.done = False
            for op in g.ops:
                if isinstance(op, FuseOp) and op.detach:
                    continue
                for r in op.inputs():
                    if r.buf.needs_grad:
                        r.buf.expected[r.key()] = r.buf.expected.get(r.key(), 0) + 1
            # consumers of one buffer read the same channel region or disjoint ones (e.g. the
            # two head convs reading their halves of the stacked head output); each region's
            # gradient is flushed on its own
            for b in g.buffers:
                keys = sorted(b.expected)
                for (a0, ac), (b0, _) in zip(keys, keys[1:]):
                    assert a0 + ac <= b0, f"{b}: consumers read overlapping regions {keys}"
        self.l1_out = torch.zeros(max(1, g.n_l1), dtype=torch.float32, device=self.device)
        self.keep.append(self.l1_out)
        self.bn_splits = 1
        for op in g.ops:
            if isinstance(op, BNOp):
                d = L.BnDesc()
                d.rows = self.nf * op.x.H * op.x.W
                self.bn_splits = max(self.bn_splits, L.load().dvie_bn_partial_splits(ctypes.byref(d)))
                d.rows = self.nb * op.x.H * op.x.W
                self.bn_splits = max(self.bn_splits, L.load().dvie_bn_partial_splits(ctypes.byref(d)))
                op.stats = torch.zeros((8, op.x.c), dtype=torch.float32, device=self.device)
                self.keep.append(op.stats)
        maxc = max([op.x.c for op in g.ops if isinstance(op, BNOp)] + [4])
        self.bn_partial = torch.zeros(self.bn_splits * 2 * maxc, dtype=torch.float64, device=self.device)
        self.keep.append(self.bn_partial)

    def ptr(self, region, n0=0, grad=False):
        b = region.buf
        t = b.g if grad else b.t
        es = elem_size(t.dtype)
        return t.data_ptr() + (n0 * b.H * b.W * b.C + region.c0) * es

    # ---------------- weight packing ----------------
    def _build_pack(self):
        descs = []
        # the tensors the pack reads (static_weights plans repack only when one changed)
        self._pack_srcs = [t for lay in self.g.layers if lay.cin_p is not None
                           for t in (lay.m.weight, lay.m.bias if lay.has_bias else None) if t is not None]
        self._pack_sig = None
        for lay in self.g.layers:
            if lay.cin_p is None:
                continue
            K = lay.kh * lay.kw * lay.cin_p
            kpad = rup(K, 64)
            lay.kpad = kpad
            lay.wf = torch.zeros((lay.cout_p, kpad), dtype=self.dtype, device=self.device)
            cmap_t = torch.tensor(lay.cmap, dtype=torch.int32, device=self.device)
            lay.cmap_t = cmap_t
            self.keep += [lay.wf, cmap_t]
            ft = lay.fwd_taps()
            descs.append(self._pack_desc(lay, lay.wf, lay.cout_p, kpad, lay.cin_p, 0, ft, cmap_t))
            if lay.has_bias:
                # (a transposed conv's bias belongs to its output = the virtual conv's input)
                nbias, rows = (lay.cin, lay.cin_p) if lay.transposed else (lay.cout, lay.cout_p)
                lay.bias_p = torch.zeros(rows, dtype=torch.float32, device=self.device)
                self.keep.append(lay.bias_p)
                d = L.PackDesc()
                d.src, d.dst, d.cmap = lay.m.bias.data_ptr(), lay.bias_p.data_ptr(), None
                d.rows, d.kpad, d.c, d.mode = rows, 1, 1, 0
                d.th, d.tw, d.kh0, d.kw0, d.dkh, d.dkw = 1, 1, 0, 0, 1, 1
                d.cout_s, d.cin_s, d.kh_s, d.kw_s, d.dtype = nbias, 1, 1, 1, L.F32
                descs.append(d)
            lay.wd = []
            lay.wd4 = None  # (the one-launch stride-2 data-gradient weights: packed by this plan)
        self._pack_descs = descs  # dgrad packs appended during backward build

    def _pack_desc(self, lay, dst, rows, kpad, c, mode, taps, cmap_t):
        if isinstance(lay.m, StackedConv):
            assert lay.m.contiguous(), f"{lay.name}: stacked parts are not consecutive in memory"
        d = L.PackDesc()
        d.src, d.dst, d.cmap = lay.m.weight.data_ptr(), dst.data_ptr(), cmap_t.data_ptr()
        d.rows, d.kpad, d.c, d.mode = rows, kpad, c, mode
        d.th, d.tw, d.kh0, d.kw0, d.dkh, d.dkw = taps["th"], taps["tw"], taps["kh0"], taps["kw0"], taps["dkh"], taps["dkw"]
        d.cout_s, d.cin_s, d.kh_s, d.kw_s, d.dtype = lay.cout, lay.cin, lay.kh, lay.kw, self.dt
        return d

    def _dgrad_weights(self, lay, H, W):
        """packed [cin_p][kpad] weights for each stride phase (cached per layer/shape)."""
        key = (H, W)
        for k, v in lay.wd:
            if k == key:
                return v
        out = []
        for ph in lay.dgrad_phases(H, W):
            kpad = rup(ph["th"] * ph["tw"] * lay.cout_p, 64)
            t = torch.zeros((lay.cin_p, kpad), dtype=self.dtype, device=self.device)
            self.keep.append(t)
            self._pack_descs.append(self._pack_desc(lay, t, lay.cin_p, kpad, lay.cout_p, 1, ph, lay.cmap_t))
            out.append((ph, t, kpad))
        lay.wd.append((key, out))
        return out

    # phase order of the one-launch stride-2 data gradient (include/dvie.h dvie_conv_desc.phc)
    PH4_ORDER = ((0, 0), (1, 1), (0, 1), (1, 0))

    def _ph4_eligible(self, lay, x):
        """stride-2 3x3 pad-1 data gradient as ONE launch of the halo kernel with the four
        output phases as channel blocks (bf16; DVIE_PH4=0 keeps the four phase launches)"""
        # phc <= 128: at 256 output channels per phase (transition1.1, 256 -> 128) the four
        # launches measured faster (0.369 vs 0.532 ms/step: each 128-channel tile of the one
        # launch streams the weight rows of all four taps, 7 of 16 of them zero for its phase,
        # and re-stages the dy halo for each of the 8 channel blocks); the 64- / 128-channel
        # layers gain 0.175 ms/step together (profiles/r06d/)
        return (self.dtype == torch.bfloat16 and os.environ.get("DVIE_PH4", "1") != "0" and lay.stride == 2
                and lay.kh == 3 and lay.kw == 3 and lay.pad == 1 and lay.dil == 1 and not lay.transposed
                and x.c == lay.cin_p and lay.cin_p % 32 == 0 and lay.cin_p <= 128
                and (lay.cout_p % 64 == 0 or lay.cout_p < 64))

    def _dgrad_weights_ph4(self, lay):
        """packed [4 * cin_p][kpad] weights of the one-launch stride-2 data gradient: row block
        q = phase (a, b) = PH4_ORDER[q], tap (i, j) of the 2 x 2 grid = forward weight
        (kh, kw) = (a + 1 - 2i, b + 1 - 2j) (zero where that is outside the kernel)"""
        if getattr(lay, "wd4", None) is not None:
            return lay.wd4
        kpad = rup(4 * lay.cout_p, 64)
        t = torch.zeros((4 * lay.cin_p, kpad), dtype=self.dtype, device=self.device)
        self.keep.append(t)
        for q, (a, b) in enumerate(self.PH4_ORDER):
            taps = dict(th=2, tw=2, kh0=a + 1, kw0=b + 1, dkh=-2, dkw=-2)
            self._pack_descs.append(self._pack_desc(lay, t[q * lay.cin_p:(q + 1) * lay.cin_p], lay.cin_p, kpad,
                                                    lay.cout_p, 1, taps, lay.cmap_t))
        lay.wd4 = (t, kpad)
        return lay.wd4

    # ---------------- descriptor factories ----------------
    def _op(self, kind):
        o = L.Op()
        o.kind = kind
        return o

    def conv_desc(self, x_ptr, x_ld, n, ih, iw, c, w_ptr, kpad, cout, oh, ow, sy, sx, taps, y_ptr, y_ld, yh, yw,
                  osy=1, osx=1, ory=0, orx=0, bias=None, res=None, res_ld=0, z=None, z_ld=0, act=0, dact=0, beta=0,
                  out_f32=False):
        o = self._op(L.OP_CONV)
        d = o.u.conv
        d.x, d.w, d.y, d.bias, d.res, d.z = x_ptr, w_ptr, y_ptr, bias, res, z
        d.x_ld, d.y_ld, d.res_ld, d.z_ld = x_ld, y_ld, res_ld, z_ld
        d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, ih, iw, c, kpad, cout
        d.oh, d.ow, d.sy, d.sx = oh, ow, sy, sx
        d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = taps["th"], taps["tw"], taps["dy0"], taps["dx0"], taps["ddy"], taps["ddx"]
        d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = yh, yw, osy, osx, ory, orx
        d.act, d.dact, d.beta, d.dtype, d.out_f32 = act, dact, beta, self.dt, int(out_f32)
        d.alpha = 0.2
        return o

    def ew_desc(self, op, n, h, w, c, y_ptr, y_ld, srcs=(), res=None, res_ld=0, z=None, z_ld=0, act=0, dact=0,
                beta=0, scale=1.0):
        o = self._op(L.OP_EW)
        d = o.u.ew
        d.op, d.n, d.h, d.w, d.c = op, n, h, w, c
        d.y, d.y_ld = y_ptr, y_ld
        d.nsrc = len(srcs)
        for i, (p, ld, sh, sw) in enumerate(srcs):
            setattr(d, f"src{i}", p)
            setattr(d, f"src_ld{i}", ld)
            setattr(d, f"sh{i}", sh)
            setattr(d, f"sw{i}", sw)
        d.res, d.res_ld, d.z, d.z_ld = res, res_ld, z, z_ld
        d.act, d.dact, d.beta, d.dtype = act, dact, beta, self.dt
        d.alpha, d.scale = 0.2, scale
        # profiling meta: algorithmic bytes = output written once (+ read when accumulating),
        # residual / activation input read once, each source read once at its own resolution
        npx = n * h * w
        nbytes = self.es * c * (npx * (1 + int(bool(beta)) + int(res is not None) + int(z is not None))
                                + sum(n * sh * sw for (_, _, sh, sw) in srcs))
        o.meta = dict(cls="pointwise", name=f"ew{op} {n}x{h}x{w}x{c} src{len(srcs)}"
                      + ("+res" if res is not None else "") + ("+acc" if beta else "") + ("+z" if z is not None else ""),
                      flops=0.0, bytes=float(nbytes))
        return o

    def _part(self, part):
        if part is None:
            return 0, self.nf
        return (0 if part == 0 else self.nf // 2), self.nf // 2

    # ---------------- forward ----------------
    def _segenc_fusable(self, ops):
        if self.dtype != torch.bfloat16 or os.environ.get("DVIE_SEGENC_FUSED", "1") == "0":
            return False
        o0, o1, o2 = ops
        acts = (L.ACT_ELU, L.ACT_ELU, L.ACT_NONE)
        chans = ((24, 32), (32, 32), (32, 8))
        for op, act, (ci, co) in zip(ops, acts, chans):
            lay = op.layer
            if not (isinstance(op, ConvOp) and op.act == act and op.res is None and lay.kh == 3 and lay.kw == 3
                    and lay.stride == 1 and lay.pad == 1 and lay.dil == 1 and lay.has_bias and op.x.c == ci
                    and op.out.c == co and lay.cout_p == co):
                return False
        if not (o1.x.buf is o0.out.buf and o2.x.buf is o1.out.buf and o0.out.c0 == 0 and o1.out.c0 == 0):
            return False
        if o0.out.buf.C != 32 or o1.out.buf.C != 32 or o2.out.buf.external:
            return False
        x = o0.x
        return self.nf * x.H * x.W * x.buf.C * 2 < 0xFFFFFF00

    def _segenc_fwd(self, ops):
        o0, o1, o2 = ops
        x, nf = o0.x, self.nf
        o = self._op(L.OP_SEGENC_FWD)
        d = o.u.segenc
        d.inp, d.e1, d.e2, d.out = self.ptr(x), self.ptr(o0.out), self.ptr(o1.out), self.ptr(o2.out)
        d.in_ld, d.e1_ld, d.e2_ld, d.out_ld = x.buf.C, o0.out.buf.C, o1.out.buf.C, o2.out.buf.C
        d.w0, d.w2, d.w4 = o0.layer.wf.data_ptr(), o1.layer.wf.data_ptr(), o2.layer.wf.data_ptr()
        d.b0, d.b2, d.b4 = o0.layer.bias_p.data_ptr(), o1.layer.bias_p.data_ptr(), o2.layer.bias_p.data_ptr()
        d.n, d.h, d.w = nf, x.H, x.W
        d.kpad0, d.kpad2, d.kpad4 = o0.layer.kpad, o1.layer.kpad, o2.layer.kpad
        npx = nf * x.H * x.W
        o.meta = dict(cls="conv_fwd", name="seg_encoder (fused)",
                      flops=2.0 * npx * 9 * sum(op.layer.cout * op.layer.cin for op in ops),
                      bytes=float(self.es * npx * (x.c + 32 + 32 + 8)))
        return o

    def _build_forward(self):
        g = self.g
        nf = self.nf
        fused_first, skip = {}, set()
        # the fused forward (one dvie_segenc_fwd per encoder) is the default since its stages
        # run two 32-pixel blocks per wave: 0.316 vs 0.344 ms per step for the three convs at
        # 8x256x512 (profiles/r06/segenc_*); DVIE_SEGENC_FWD=0 runs the three convs
        fwd_on = os.environ.get("DVIE_SEGENC_FWD", "1") == "1"
        for chain in getattr(g, "segenc", []) if fwd_on else []:
            if self._segenc_fusable(chain):
                fused_first[id(chain[0])] = chain
                skip.update(id(op) for op in chain[1:])
        for op in g.ops:
            if id(op) in skip:
                continue
            if id(op) in fused_first:
                self.fwd.append(self._segenc_fwd(fused_first[id(op)]))
                continue
            if isinstance(op, InputOp):
                n0, cnt = self._part(op.part)
                o = self.ew_desc(L.EW_NCHW, cnt, op.out.H, op.out.W, op.out.c, self.ptr(op.out, n0), op.out.buf.C)
                o.u.ew.ext_c = op.ext_c
                if op.normalize:
                    m = torch.tensor(_IMAGENET_MEAN + [0.0] * 5, dtype=torch.float32, device=self.device)
                    s = torch.tensor(_IMAGENET_STD + [1.0] * 5, dtype=torch.float32, device=self.device)
                    self.keep += [m, s]
                    o.u.ew.mean, o.u.ew.std = m.data_ptr(), s.data_ptr()
                    op.std_t = s
                self.ext_in.setdefault(op.key, []).append((len(self.fwd), op))
                self.fwd.append(o)
            elif isinstance(op, ConvOp):
                lay, x, out = op.layer, op.x, op.out
                ext = out.buf.external
                o = self.conv_desc(
                    self.ptr(x), x.buf.C, nf, x.H, x.W, x.c, lay.wf.data_ptr(), lay.kpad, lay.cout_p, out.H, out.W,
                    lay.stride, lay.stride, lay.fwd_taps(), 0 if ext else self.ptr(out), out.buf.C, out.H, out.W,
                    bias=lay.bias_p.data_ptr() if lay.has_bias else None,
                    res=self.ptr(op.res) if op.res is not None else None,
                    res_ld=op.res.buf.C if op.res is not None else 0, act=op.act,
                    out_f32=(out.buf.dt == torch.float32 and self.dtype != torch.float32))
                npx = nf * out.H * out.W
                o.meta = dict(cls="conv_fwd", name=lay.name,
                              flops=2.0 * npx * lay.cout * lay.cin * lay.kh * lay.kw,
                              bytes=float(self.es * (nf * x.H * x.W * lay.cin + npx * lay.cout * (2 if op.res is not None else 1)
                                                     + lay.cout * lay.cin * lay.kh * lay.kw)))
                if ext:
                    self.ext_out.setdefault(out.buf.name, []).append((len(self.fwd), out))
                self.fwd.append(o)
            elif isinstance(op, ConvTOp):
                # the stride phases of the virtual conv's data gradient, over the ConvT input
                lay, x, out = op.layer, op.x, op.out
                assert not out.buf.external
                for ph, wt, kpad in self._dgrad_weights(lay, out.H, out.W):
                    o = self.conv_desc(
                        self.ptr(x), x.buf.C, nf, x.H, x.W, lay.cout_p, wt.data_ptr(), kpad, out.c, ph["oh"], ph["ow"],
                        1, 1, ph, self.ptr(out), out.buf.C, out.H, out.W, osy=lay.stride, osx=lay.stride,
                        ory=ph["ry"], orx=ph["rx"], bias=lay.bias_p.data_ptr() if lay.has_bias else None, act=op.act,
                        out_f32=(out.buf.dt == torch.float32 and self.dtype != torch.float32))
                    npx = nf * ph["oh"] * ph["ow"]
                    o.meta = dict(cls="conv_fwd", name=lay.name, flops=2.0 * npx * lay.cout * lay.cin * ph["th"] * ph["tw"],
                                  bytes=float(self.es * (nf * x.H * x.W * lay.cout + npx * lay.cin)))
                    self.fwd.append(o)
            elif isinstance(op, AttnOp):
                self.fwd.append(self._attn_fwd(op))
            elif isinstance(op, FuseOp):
                out = op.out
                srcs = [(self.ptr(s), s.buf.C, s.H, s.W) for s in op.srcs]
                o = self.ew_desc(L.EW_FUSE, nf, out.H, out.W, out.c, self.ptr(out), out.buf.C, srcs, act=op.act)
                o.u.ew.align = int(op.align)
                self.fwd.append(o)
            elif isinstance(op, MaskOp):
                out, src = op.out, op.src
                o = self.ew_desc(L.EW_MASK, nf, out.H, out.W, out.c, self.ptr(out), out.buf.C,
                                 [(self.ptr(src), src.buf.C, src.H, src.W)])
                o.u.ew.ext_c = int(op.inverse)
                self.ext_mask = getattr(self, "ext_mask", {})
                self.ext_mask.setdefault(op.key, []).append(("fwd", len(self.fwd), op))
                self.fwd.append(o)
            elif isinstance(op, OutNCHWOp):
                r = op.region
                o = self.ew_desc(L.EW_TONCHW, nf, r.H, r.W, r.c, 0, 0, [(self.ptr(r), r.buf.C, r.H, r.W)])
                o.u.ew.ext_c = op.channels
                self.ext_nchw_out = getattr(self, "ext_nchw_out", {})
                self.ext_nchw_out[op.key] = len(self.fwd)
                self.fwd.append(o)
            elif isinstance(op, PoolOp):
                x, out = op.x, op.out
                self.fwd.append(self.ew_desc(L.EW_POOL, nf, out.H, out.W, out.c, self.ptr(out), out.buf.C,
                                             [(self.ptr(x), x.buf.C, x.H, x.W)]))
            elif isinstance(op, BNOp):
                o = self._op(L.OP_BN_FWD)
                self._bn_common(o.u.bn, op, nf)
                o.u.bn.y, o.u.bn.y_ld = self.ptr(op.out), op.out.buf.C
                op.fwd_index = len(self.fwd)
                self.bn_ops = getattr(self, "bn_ops", []) + [op]
                self.fwd.append(o)
            elif isinstance(op, HeadOp):
                x = op.x
                o = self._op(L.OP_HEAD_FWD)
                d = o.u.head
                d.x, d.x_ld = self.ptr(x), x.buf.C
                d.n, d.h, d.w, d.c, d.pool, d.dtype = nf, x.H, x.W, x.c, op.pool, self.dt
                rows = nf * (x.H // op.pool) * (x.W // op.pool)
                op.pooled = torch.zeros(rows * x.c, dtype=torch.float32, device=self.device)
                self.keep.append(op.pooled)
                d.pooled = op.pooled.data_ptr()
                self.ext_head = getattr(self, "ext_head", {})
                self.ext_head[op.key] = (len(self.fwd), rows)
                self.fwd.append(o)
            elif isinstance(op, L1FeatOp):
                a = op.a
                half = nf // 2
                o = self._op(L.OP_LOSS)
                d = o.u.loss
                d.a, d.b = self.ptr(a, 0), self.ptr(a, half)
                sn, sh, sw = a.H * a.W * a.buf.C, a.W * a.buf.C, a.buf.C
                d.a_sn, d.a_sc, d.a_sh, d.a_sw = sn, 1, sh, sw
                d.b_sn, d.b_sc, d.b_sh, d.b_sw = sn, 1, sh, sw
                d.kind, d.bsz, d.ch, d.h, d.w, d.dtype = L.LOSS_L1NHWC, half, a.c, a.H, a.W, self.dt
                d.weight, d.out_scale = 1.0, 1.0
                npart = L.load().dvie_loss_partial_count(ctypes.byref(d))
                part = torch.zeros(max(1, npart), dtype=torch.float64, device=self.device)
                self.keep.append(part)
                d.partial = part.data_ptr()
                d.out = self.l1_out.data_ptr() + 4 * op.idx
                self._l1_fwd.append((len(self.fwd), op.idx))
                self.fwd.append(o)
            else:
                raise TypeError(op)

    # ---------------- local-window attention ----------------
    _ATTN_FWD = {"l2norm": L.ATTN_L2NORM, "corr": L.ATTN_CORR, "softmax": L.ATTN_SOFTMAX, "wnorm": L.ATTN_WNORM,
                 "gather": L.ATTN_GATHER, "pool": L.ATTN_POOL}

    def attn_desc(self, kind, n, region_hw, c, a, a_ld, y, y_ld, b0=None, b1=None, b_ld=0, wh=1, ww=1, nhalf=1,
                  half0=0, res=None, res_ld=0, z=None, z_ld=0, dact=0, beta=0):
        o = self._op(L.OP_ATTN)
        d = o.u.attn
        d.op, d.n, d.h, d.w, d.c = kind, n, region_hw[0], region_hw[1], c
        d.a, d.a_ld, d.y, d.y_ld, d.b0, d.b1, d.b_ld = a, a_ld, y, y_ld, b0, b1, b_ld
        d.wh, d.ww, d.nhalf, d.half0 = wh, ww, nhalf, half0
        d.res, d.res_ld, d.z, d.z_ld, d.dact, d.beta = res, res_ld, z, z_ld, dact, beta
        d.dtype, d.alpha = self.dt, 0.2
        return o

    def _attn_fwd(self, op):
        a, out = op.a, op.out
        bs = [self.ptr(b) for b in op.bs] + [None, None]
        b_ld = op.bs[0].buf.C if op.bs else 0
        if len(op.bs) == 2:
            assert op.bs[1].buf.C == b_ld, "attn: target maps need one pixel stride"
        o = self.attn_desc(self._ATTN_FWD[op.kind], self.nf, (out.H, out.W), op.c, self.ptr(a), a.buf.C,
                           self.ptr(out), out.buf.C, bs[0], bs[1], b_ld, op.wh, op.ww, op.nhalf, op.half0)
        npx = self.nf * out.H * out.W
        o.meta = dict(cls="attn", name=f"{op.kind}:{out.buf.name}", flops=0.0,
                      bytes=float(self.es * npx * (a.c + sum(b.c for b in op.bs) + out.c)))
        return o

    def _attn_backward(self, op, gout, gld):
        """Gradient contributions of one attention op (formulas in include/dvie.h)."""
        nb = self.nb
        a, out = op.a, op.out
        hw = (out.H, out.W)
        K = op.wh * op.ww
        ld_a = a.buf.C

        npx = nb * out.H * out.W
        J = op.nhalf * K
        cb = sum(b.c for b in op.bs)
        # algorithmic channels touched per pixel by each backward kernel (profiling meta):
        # its reads (upstream gradient, saved operands) and its written gradient
        moved = {"l2norm": 4 * op.c, "softmax": 3 * J, "wnorm": 4 * J, "pool": 2 * op.c,
                 "corr": op.c + J + cb, "gather": out.c + J + cb}[op.kind]

        def contrib(region, build):
            if region.buf.needs_grad:
                def emit(beta, res, res_ld, dact, z, z_ld):
                    o = build(dict(res=res, res_ld=res_ld, dact=dact, z=z, z_ld=z_ld, beta=beta))
                    o.meta = dict(cls="attn_bwd", name=f"{op.kind}:{region.buf.name}", flops=0.0,
                                  bytes=float(self.es * npx * moved))
                    return [o]
                self._contrib(region, emit)

        if op.kind == "l2norm":  # a = x, out = x / |x|
            contrib(a, lambda e: self.attn_desc(L.ATTN_L2NORM_BWD, nb, hw, op.c, gout, gld, self.ptr(a, grad=True),
                                                ld_a, self.ptr(out), self.ptr(a), self._same_ld(out, a), **e))
        elif op.kind == "softmax":
            contrib(a, lambda e: self.attn_desc(L.ATTN_SOFTMAX_BWD, nb, hw, op.c, gout, gld, self.ptr(a, grad=True),
                                                ld_a, self.ptr(out), None, out.buf.C, op.wh, op.ww, op.nhalf, **e))
        elif op.kind == "wnorm":
            contrib(a, lambda e: self.attn_desc(L.ATTN_WNORM_BWD, nb, hw, op.c, gout, gld, self.ptr(a, grad=True),
                                                ld_a, self.ptr(out), self.ptr(a), self._same_ld(out, a), op.wh,
                                                op.ww, op.nhalf, **e))
        elif op.kind == "pool":
            contrib(a, lambda e: self.attn_desc(L.ATTN_POOL_T, nb, hw, op.c, gout, gld, self.ptr(a, grad=True), ld_a,
                                                wh=op.wh, ww=op.ww, **e))
        elif op.kind == "corr":  # S[p, m*K+k] = <a(p), b_m(p+o_k)>
            bs = op.bs
            bp = [self.ptr(b) for b in bs] + [None]
            contrib(a, lambda e: self.attn_desc(L.ATTN_GATHER, nb, hw, op.c, gout, gld, self.ptr(a, grad=True), ld_a,
                                                bp[0], bp[1], bs[0].buf.C, op.wh, op.ww, op.nhalf, 0, **e))
            for m, b in enumerate(bs):
                contrib(b, lambda e, m=m, b=b: self.attn_desc(
                    L.ATTN_GATHER_T, nb, hw, op.c, gout, gld, self.ptr(b, grad=True), b.buf.C, self.ptr(a), None,
                    ld_a, op.wh, op.ww, op.nhalf, m, **e))
        elif op.kind == "gather":  # out(p) = sum_m sum_k a[p, (half0+m)K + k] f_m(p + o_k)
            fs = op.bs
            maps = [None] * op.nhalf
            for m, f in enumerate(fs):
                maps[op.half0 + m] = self.ptr(f)
            assert op.nhalf <= 2
            maps += [None]
            contrib(a, lambda e: self.attn_desc(L.ATTN_CORR, nb, hw, out.c, gout, gld, self.ptr(a, grad=True), ld_a,
                                                maps[0], maps[1], fs[0].buf.C, op.wh, op.ww, op.nhalf, **e))
            for m, f in enumerate(fs):
                contrib(f, lambda e, m=m, f=f: self.attn_desc(
                    L.ATTN_GATHER_T, nb, hw, out.c, self.ptr(a), ld_a, self.ptr(f, grad=True), f.buf.C, gout, None,
                    gld, op.wh, op.ww, op.nhalf, op.half0 + m, **e))
        else:
            raise TypeError(op.kind)

    @staticmethod
    def _same_ld(r0, r1):
        assert r0.buf.C == r1.buf.C, f"attn backward: {r0.buf} and {r1.buf} need one pixel stride"
        return r0.buf.C

    def _bn_common(self, d, op, n):
        x, m = op.x, op.m
        d.x, d.x_ld = self.ptr(x), x.buf.C
        d.rows, d.c = n * x.H * x.W, x.c
        d.splits = L.load().dvie_bn_partial_splits(ctypes.byref(d))
        d.partial, d.stats = self.bn_partial.data_ptr(), op.stats.data_ptr()
        d.gamma = m.weight.data_ptr() if m.weight is not None else None
        d.beta = m.bias.data_ptr() if m.bias is not None else None
        d.running_mean = m.running_mean.data_ptr() if m.running_mean is not None else None
        d.running_var = m.running_var.data_ptr() if m.running_var is not None else None
        assert m.num_features == x.c or rup(m.num_features, PADC) == x.c
        assert m.num_features == x.c, "BatchNorm channel count must be a multiple of 8"
        d.training = int(getattr(self.g, "bn_training", True))
        d.act, d.alpha, d.eps = op.act, 0.2, m.eps
        d.x_f32 = int(x.buf.dt == torch.float32 and self.dtype != torch.float32)
        d.momentum = m.momentum if m.momentum is not None else 0.0
        d.dtype = self.dt

    # ---------------- backward ----------------
    def _contrib(self, region, emitter, ident=None):
        """Record a gradient contribution to `region`'s buffer: either a kernel
        (emitter(beta, res_ptr, res_ld, dact, z_ptr, z_ld) -> ops) or an identity
        (`ident` = (ptr, ld) of a gradient region with the same shape)."""
        b = region.buf
        key = region.key()
        assert key in b.expected, (b, key)
        pend = b.pending.setdefault(key, [])
        pend.append((emitter, ident))
        if len(pend) == b.expected[key]:
            self._flush(b, key)

    def _flush(self, b, key):
        c0, c = key
        region = Region(b, c0, c)
        pending = b.pending.pop(key)
        kernels = [e for e, i in pending if e is not None]
        idents = [i for e, i in pending if e is None]
        prod = b.producers
        # the producer's activation derivative rides on the last contribution of each region
        # when one activated producer wrote the buffer and the read regions tile its output
        # exactly (else _ensure_dact applies it in a pass of its own)
        fuse_dact = False
        if len(prod) == 1 and prod[0].act != L.ACT_NONE and prod[0].out.buf is b:
            o0, oc = prod[0].out.c0, prod[0].out.c
            fuse_dact = (all(o0 <= k0 and k0 + kc <= o0 + oc for k0, kc in b.expected) and
                         sum(kc for _, kc in b.expected) == oc)
        b.dact_done = fuse_dact
        dact = prod[0].act if fuse_dact else 0
        z = self.ptr(region) if fuse_dact else None
        if fuse_dact:
            assert b.dt == self.dtype
        seq = []
        k = 0
        for em in kernels:
            r = idents[k] if k < len(idents) else None
            k += 1 if r is not None else 0
            seq.append((em, r))
        rest = idents[k:]
        gptr, gld = self.ptr(region, grad=True), b.C
        while rest:
            a = rest.pop(0)
            r = rest.pop(0) if rest else None

            def copy_em(beta, res, res_ld, dact_, z_, z_ld_, a=a):
                return [self.ew_desc(L.EW_COPY, self.nb, b.H, b.W, c, gptr, gld, [(a[0], a[1], b.H, b.W)],
                                     res=res, res_ld=res_ld, z=z_, z_ld=z_ld_, dact=dact_, beta=beta)]

            seq.append((copy_em, r))
        for i, (em, r) in enumerate(seq):
            last = i == len(seq) - 1
            ops = em(0 if i == 0 else 1, r[0] if r else None, r[1] if r else 0, dact if last else 0,
                     z if last else None, b.C if last else 0)
            self.bwd.extend(ops)
        b.n_flushed += 1
        b.done = b.n_flushed == len(b.expected)

    def _ensure_dact(self, op):
        """Producer-side activation derivative when it could not be fused upstream."""
        b = op.out.buf
        if op.act == L.ACT_NONE or getattr(b, "dact_done", False):
            return
        out = op.out
        gp = self.ptr(out, grad=True)
        self.bwd.append(self.ew_desc(L.EW_COPY, self.nb, out.H, out.W, out.c, gp, b.C, [(gp, b.C, out.H, out.W)],
                                     z=self.ptr(out), z_ld=b.C, dact=op.act))

    def _segenc_bwd_chains(self):
        """id(last op) -> chain for the segmentation encoders whose backward runs as one
        dvie_segenc_bwd launch: the forward is fusable, the encoder input needs no gradient and
        the intermediates have no other reader."""
        out = {}
        if os.environ.get("DVIE_SEGENC_FUSED", "1") == "0":
            return out
        for chain in getattr(self.g, "segenc", []):
            o0, o1, o2 = chain
            if not self._segenc_fusable(chain) or o0.x.buf.needs_grad:
                continue
            if not all(op.layer.trainable for op in chain):
                continue
            if len(o0.out.buf.consumers) != 1 or len(o1.out.buf.consumers) != 1:
                continue
            if self.nb * o0.x.H * o0.x.W * max(o2.out.buf.C, 32) * 2 >= 0xFFFFFF00:
                continue
            out[id(o2)] = chain
        return out

    def _segenc_backward(self, chain, gout, gld):
        """dvie_segenc_bwd (all three weight / bias gradients of one encoder, d_e2 and d_e1 on
        chip) into this chain's own slab buffers, then the slab reductions on the weight lane."""
        o0, o1, o2 = chain
        x, nb = o0.x, self.nb
        slabs = 256
        bufs = {k: torch.empty(slabs * n, dtype=torch.float32, device=self.device) for k, n in
                (("dw4", 8 * 288), ("dw2", 32 * 288), ("dw0", 32 * 216), ("db4", 8), ("db2", 32), ("db0", 32))}
        self.keep += list(bufs.values())
        (_, w4d, kpad4), = self._dgrad_weights(o2.layer, x.H, x.W)
        (_, w2d, kpad2), = self._dgrad_weights(o1.layer, x.H, x.W)
        o = self._op(L.OP_SEGENC_BWD)
        d = o.u.segenc_bwd
        d.dout, d.e2, d.e1, d.inp = gout, self.ptr(o1.out), self.ptr(o0.out), self.ptr(x)
        d.dout_ld, d.e2_ld, d.e1_ld, d.in_ld = gld, o1.out.buf.C, o0.out.buf.C, x.buf.C
        d.w4d, d.w2d, d.kpad4, d.kpad2 = w4d.data_ptr(), w2d.data_ptr(), kpad4, kpad2
        for k in ("dw4", "dw2", "dw0", "db4", "db2", "db0"):
            setattr(d, k, bufs[k].data_ptr())
        d.n, d.h, d.w, d.slabs = nb, x.H, x.W, slabs
        npx = nb * x.H * x.W
        o.meta = dict(cls="conv_wgrad", name="seg_encoder (fused backward)",
                      flops=2.0 * npx * 9 * (2 * o2.layer.cout * o2.layer.cin + 2 * o1.layer.cout * o1.layer.cin
                                             + o0.layer.cout * o0.layer.cin),
                      bytes=float(self.es * npx * (8 + 32 + 32 + x.c)))
        self.bwd.append(o)
        for op, wk, bk in ((o2, "dw4", "db4"), (o1, "dw2", "db2"), (o0, "dw0", "db0")):
            lay, xin = op.layer, op.x
            first = lay not in self.wg_first
            r_op = self._op(L.OP_WREDUCE)
            r = r_op.u.wreduce
            r.ws, r.dw, r.cmap = bufs[wk].data_ptr(), 0, lay.cmap_t.data_ptr()
            r.splits, r.ws_rows, r.ws_k, r.co_off = slabs, lay.cout_p, 9 * xin.c, 0
            r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, lay.cin, lay.kh, lay.kw, xin.c
            r.beta = 0 if first else 1
            r_op.ws_ptr = bufs[wk].data_ptr()
            r_op.meta = _reduce_meta(lay.name, r)
            self.bwd.append(r_op)
            self._grad_slots.append((len(self.bwd) - 1, lay, "weight", first))
            b_op = self._op(L.OP_WREDUCE)
            r = b_op.u.wreduce
            r.ws, r.dw, r.cmap = bufs[bk].data_ptr(), 0, None
            r.splits, r.ws_rows, r.ws_k, r.co_off = slabs, lay.cout_p, 1, 0
            r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, 1, 1, 1, 1
            r.beta = 0 if first else 1
            b_op.ws_ptr = bufs[bk].data_ptr()
            b_op.meta = _reduce_meta(lay.name + ".bias", r)
            self.bwd.append(b_op)
            self._grad_slots.append((len(self.bwd) - 1, lay, "bias", first))
            self.wg_first[lay] = True
            self._uses_left[lay] -= 1
            if self._uses_left[lay] == 0:
                self.completions.append((len(self.bwd), lay))
        for op in (o0, o1):  # their output gradients are never formed (d_e1 / d_e2 stay on chip)
            op.out.buf.done = True
            op.out.buf.dact_done = True
            op.out.buf.pending = {}

    def _build_backward(self):
        g = self.g
        nb = self.nb
        seg_bwd = self._seg_bwd
        seg_skip = {id(op) for ch in seg_bwd.values() for op in ch[:2]}
        self.wg_first = {}
        self.completions = []  # (bwd index, layer): the layer's parameter gradients are final
        self._uses_left = {}
        for op in g.ops:
            if isinstance(op, (ConvOp, ConvTOp)) and op.layer.trainable:
                self._uses_left[op.layer] = self._uses_left.get(op.layer, 0) + 1
        for key, (region, ch) in g.outputs.items():
            b = region.buf
            assert b.needs_grad and not b.expected
            assert b.t is not None or all(p.act == L.ACT_NONE for p in b.producers), "external output with activation"
            o = self.ew_desc(L.EW_NCHW, nb, region.H, region.W, region.c, self.ptr(region, grad=True), b.C)
            o.u.ew.ext_c = ch
            self.ext_ograd[key] = len(self.bwd)
            self.bwd.append(o)
            b.done = True
            b.dact_done = all(p.act == L.ACT_NONE for p in b.producers)  # else _ensure_dact at the producer
        for op in reversed(g.ops):
            if isinstance(op, OutNCHWOp):
                continue
            if isinstance(op, HeadOp):
                x = op.x
                if not x.buf.needs_grad:
                    continue
                xg = self.ptr(x, grad=True)

                def em(beta, res, res_ld, dact, z, z_ld, op=op, x=x, xg=xg):
                    assert res is None and dact == 0, "head backward has no fused epilogue"
                    o = self._op(L.OP_HEAD_BWD)
                    d = o.u.head
                    d.gx, d.gx_ld = xg, x.buf.C
                    d.n, d.h, d.w, d.c, d.pool, d.dtype, d.beta = nb, x.H, x.W, x.c, op.pool, self.dt, beta
                    self.ext_head_grad = getattr(self, "ext_head_grad", {})
                    self.ext_head_grad[op.key] = len(self.bwd)
                    return [o]

                self._contrib(x, em)
                continue
            if isinstance(op, L1FeatOp):
                a = op.a
                if not a.buf.needs_grad:
                    continue
                numel = (self.nf // 2) * a.H * a.W * a.c
                ap, bp, ld = self.ptr(a, 0), self.ptr(a, self.nf // 2), a.buf.C
                gp = self.ptr(a, grad=True)
                scale = op.weight / numel

                def em(beta, res, res_ld, dact, z, z_ld, a=a, ap=ap, bp=bp, ld=ld, gp=gp, scale=scale):
                    o = self.ew_desc(L.EW_L1SIGN, nb, a.H, a.W, a.c, gp, ld, [(ap, ld, a.H, a.W), (bp, ld, a.H, a.W)],
                                     res=res, res_ld=res_ld, z=z, z_ld=z_ld, dact=dact, beta=beta, scale=scale)
                    o.l1_seed = scale  # set_l1_loss rescales the seeds of the backward
                    return [o]

                self._contrib(a, em)
                continue
            out = op.out
            b = out.buf
            if not b.needs_grad or not getattr(b, "done", False):
                continue  # no gradient reaches this op
            if id(op) in seg_skip:
                continue  # inside a fused encoder backward: its gradient is never formed
            self._ensure_dact(op)
            gout, gld = self.ptr(out, grad=True), b.C
            if isinstance(op, InputOp):
                if op.requires_grad:
                    o = self.ew_desc(L.EW_TONCHW, nb, out.H, out.W, out.c, 0, 0, [(gout, gld, out.H, out.W)])
                    o.u.ew.ext_c = op.ext_c
                    if op.normalize:
                        o.u.ew.std = op.std_t.data_ptr()
                    self.ext_grad.setdefault(op.key, []).append((len(self.bwd), op))
                    self.bwd.append(o)
                continue
            if id(op) in seg_bwd:
                self._segenc_backward(seg_bwd[id(op)], gout, gld)
                continue
            if isinstance(op, ConvOp):
                self._conv_backward(op, gout, gld)
            elif isinstance(op, ConvTOp):
                self._convT_backward(op, gout, gld)
            elif isinstance(op, BNOp):
                x = op.x
                assert len(x.buf.consumers) == 1, "BatchNorm input must have no other reader"
                xg = self.ptr(x, grad=True) if x.buf.needs_grad else None
                if x.buf.needs_grad:
                    def em(beta, res, res_ld, dact, z, z_ld, op=op, x=x, xg=xg, gout=gout, gld=gld):
                        assert res is None and dact == 0, "BatchNorm backward has no fused epilogue"
                        o = self._op(L.OP_BN_BWD)
                        d = o.u.bn
                        self._bn_common(d, op, nb)
                        d.g, d.g_ld = gout, gld
                        d.dx, d.dx_ld, d.beta_dx = xg, x.buf.C, beta
                        if op.trainable:
                            self._grad_slots.append((len(self.bwd), op.m, "bn", op.m not in self.wg_first))
                            self.wg_first[op.m] = True
                        return [o]

                    self._contrib(x, em)
            elif isinstance(op, AttnOp):
                self._attn_backward(op, gout, gld)
            elif isinstance(op, FuseOp):
                if op.detach:
                    continue
                for s in op.srcs:
                    if not s.buf.needs_grad:
                        continue
                    if (s.H, s.W) == (out.H, out.W):
                        self._contrib(s, None, ident=(gout, gld))
                    else:
                        sp = self.ptr(s, grad=True)

                        def em(beta, res, res_ld, dact, z, z_ld, s=s, sp=sp, out=out, gout=gout, gld=gld, op=op):
                            o = self.ew_desc(L.EW_UPT, nb, s.H, s.W, s.c, sp, s.buf.C, [(gout, gld, out.H, out.W)],
                                             res=res, res_ld=res_ld, z=z, z_ld=z_ld, dact=dact, beta=beta)
                            o.u.ew.align = int(op.align)
                            return [o]

                        self._contrib(s, em)
            elif isinstance(op, MaskOp):
                src = op.src
                if src.buf.needs_grad:
                    sp = self.ptr(src, grad=True)

                    def em(beta, res, res_ld, dact, z, z_ld, src=src, sp=sp, out=out, gout=gout, gld=gld, op=op):
                        o = self.ew_desc(L.EW_MASK, nb, src.H, src.W, src.c, sp, src.buf.C, [(gout, gld, out.H, out.W)],
                                         res=res, res_ld=res_ld, z=z, z_ld=z_ld, dact=dact, beta=beta)
                        o.u.ew.ext_c = int(op.inverse)
                        self.ext_mask = getattr(self, "ext_mask", {})
                        self.ext_mask.setdefault(op.key, []).append(("bwd", len(self.bwd), op))
                        return [o]

                    self._contrib(src, em)
            elif isinstance(op, PoolOp):
                x = op.x
                if x.buf.needs_grad:
                    xp = self.ptr(x, grad=True)

                    def em(beta, res, res_ld, dact, z, z_ld, x=x, xp=xp, out=out, gout=gout, gld=gld):
                        return [self.ew_desc(L.EW_POOLT, nb, x.H, x.W, x.c, xp, x.buf.C, [(gout, gld, out.H, out.W)],
                                             res=res, res_ld=res_ld, z=z, z_ld=z_ld, dact=dact, beta=beta)]

                    self._contrib(x, em)
        # (buffers whose contributions never completed would indicate a graph bug)
        for bf in g.buffers:
            if bf.needs_grad and bf.expected and not getattr(bf, "done", False):
                raise RuntimeError(f"incomplete gradient for {bf}: pending {({k: len(v) for k, v in bf.pending.items()})}"
                                   f" of {bf.expected}")

    def _head3_fusable(self, op, gld):
        """Narrow-output 3x3 head conv (HRNet rgb_layer[2] / seg_layer[2]) whose backward can
        run as one dvie_head3_bwd pass over its input.  DVIE_HEAD3_FUSED: 1 (default) the rgb
        head (8 padded channels) only -- measured 0.905 -> 0.655 ms per step, while the fused
        seg head (24) ran 1.274 ms against 1.059 unfused (profiles/r04e/ops.txt); 2 both; 0 none."""
        lay, x, out = op.layer, op.x, op.out
        mode = os.environ.get("DVIE_HEAD3_FUSED", "1")
        if self.dtype != torch.bfloat16 or mode == "0" or (mode == "1" and lay.cout_p != 8):
            return False
        if os.environ.get("DVIE_IM2COL_DGRAD", "0") == "1":  # the opt-in im2col lowering asked for
            return False
        if not (lay.trainable and x.buf.needs_grad and op.res is None and lay.kh == 3 and lay.kw == 3
                and lay.stride == 1 and lay.pad == 1 and lay.dil == 1 and lay.cout_p in (8, 24)
                and x.c % 64 == 0 and (out.H, out.W) == (x.H, x.W)):
            return False
        if x.buf.expected.get(x.key(), 0) != 1 or lay.cmap_t is not None and lay.cin != x.c:
            return False
        npx = self.nb * x.H * x.W
        return npx * max(x.buf.C, gld) * 2 < 0xFFFFFF00

    def _head3_ops(self, op, gout, gld, phase, xg, dact):
        """dvie_head3_bwd (data gradient with act' + weight-gradient slabs in one pass over
        the input) into its own slab buffer, then on the weight lane the bias column sums and
        the slab reductions; the weight-gradient bookkeeping of _emit_wgrad."""
        lay, x, out = op.layer, op.x, op.out
        nb = self.nb
        ph, wt, kpad = phase
        n_cb = x.c // 64
        splits = max(1, 256 // n_cb)
        slabs = torch.empty(splits * lay.cout_p * 9 * x.c, dtype=torch.float32, device=self.device)
        self.keep.append(slabs)
        o = self._op(L.OP_HEAD3_BWD)
        d = o.u.head3
        d.g, d.h, d.wd, d.dh, d.ws = gout, self.ptr(x), wt.data_ptr(), xg, slabs.data_ptr()
        d.g_ld, d.h_ld, d.dh_ld = gld, x.buf.C, x.buf.C
        d.n, d.hgt, d.wid, d.c = nb, x.H, x.W, x.c
        d.cout, d.kpad, d.dy0, d.dx0 = lay.cout_p, kpad, ph["dy0"], ph["dx0"]
        d.splits, d.dact, d.alpha = splits, dact, 0.2
        npix = nb * x.H * x.W
        o.meta = dict(cls="conv_dgrad", name=lay.name + "+wgrad",
                      flops=2.0 * npix * lay.cout * lay.cin * 9 * 2,
                      bytes=float(self.es * (2 * npix * x.c + npix * lay.cout) + 4 * slabs.numel()))
        ops = [o]
        first = lay not in self.wg_first
        base = len(self.bwd)
        if lay.has_bias:
            csplits = max(1, min(2048, npix // 512))
            c = self._op(L.OP_COLSUM)
            cd = c.u.colsum
            cd.g, cd.ws, cd.g_ld, cd.rows, cd.c, cd.splits, cd.dtype = gout, 0, gld, npix, lay.cout_p, csplits, self.dt
            self.ws_floats = max(self.ws_floats, csplits * lay.cout_p)
            ops.append(c)
        r_op = self._op(L.OP_WREDUCE)
        r = r_op.u.wreduce
        r.ws, r.dw, r.cmap = slabs.data_ptr(), 0, lay.cmap_t.data_ptr()
        r.splits, r.ws_rows, r.ws_k, r.co_off = splits, lay.cout_p, 9 * x.c, 0
        r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, lay.cin, lay.kh, lay.kw, x.c
        r.beta = 0 if first else 1
        r_op.ws_ptr = slabs.data_ptr()
        r_op.meta = _reduce_meta(lay.name, r)
        ops.append(r_op)
        self._grad_slots.append((base + len(ops) - 1, lay, "weight", first))
        if lay.has_bias:
            b_op = self._op(L.OP_WREDUCE)
            r = b_op.u.wreduce
            r.ws, r.dw, r.cmap = 0, 0, None
            r.splits, r.ws_rows, r.ws_k, r.co_off = csplits, lay.cout_p, 1, 0
            r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, 1, 1, 1, 1
            r.beta = 0 if first else 1
            b_op.meta = _reduce_meta(lay.name + ".bias", r)
            ops.append(b_op)
            self._grad_slots.append((base + len(ops) - 1, lay, "bias", first))
        self.wg_first[lay] = True
        self._uses_left[lay] -= 1
        if self._uses_left[lay] == 0:
            self.completions.append((base + len(ops), lay))
        return ops

    def _conv_backward(self, op, gout, gld):
        lay, x, out = op.layer, op.x, op.out
        nb = self.nb
        npix = nb * out.H * out.W
        taps = lay.fwd_taps()
        head3 = self._head3_fusable(op, gld)
        if lay.trainable and not head3:
            self._emit_wgrad(op, gout, gld)
        if op.res is not None and op.res.buf.needs_grad:
            self._contrib(op.res, None, ident=(gout, gld))
        if x.buf.needs_grad:
            phases = self._dgrad_weights(lay, x.H, x.W)
            xg = self.ptr(x, grad=True)

            def em(beta, res, res_ld, dact, z, z_ld, phases=phases, x=x, xg=xg, out=out, gout=gout, gld=gld, lay=lay):
                if head3:
                    if beta == 0 and res is None and dact in (L.ACT_NONE, L.ACT_LRELU) and \
                            (z is None or z == self.ptr(x)) and len(phases) == 1:
                        return self._head3_ops(op, gout, gld, phases[0], xg, dact)
                    self._emit_wgrad(op, gout, gld)  # (not the expected pattern: unfused)
                ops = []
                if self._im2col_dgrad(lay, x, phases):
                    return self._im2col_dgrad_ops(lay, x, xg, out, gout, gld, phases[0], res, res_ld, z, z_ld, dact,
                                                  beta)
                if self._ph4_eligible(lay, x):
                    wt, kpad = self._dgrad_weights_ph4(lay)
                    taps = dict(th=2, tw=2, dy0=0, dx0=0, ddy=1, ddx=1)
                    o = self.conv_desc(gout, gld, nb, out.H, out.W, lay.cout_p, wt.data_ptr(), kpad, 4 * x.c, out.H,
                                       out.W, 1, 1, taps, xg, x.buf.C, x.H, x.W, osy=2, osx=2, res=res, res_ld=res_ld,
                                       z=z, z_ld=z_ld, dact=dact, beta=beta)
                    o.u.conv.phc = x.c
                    npx = nb * x.H * x.W
                    o.meta = dict(cls="conv_dgrad", name=lay.name,
                                  flops=2.0 * nb * out.H * out.W * lay.cin * lay.cout * 9,
                                  bytes=float(self.es * (nb * out.H * out.W * lay.cout
                                                         + npx * lay.cin * (1 + (res is not None) + (z is not None) + beta)
                                                         + lay.cout * lay.cin * 9)))
                    return [o]
                for ph, wt, kpad in phases:
                    o = self.conv_desc(
                        gout, gld, nb, out.H, out.W, lay.cout_p, wt.data_ptr(), kpad, x.c, ph["oh"], ph["ow"], 1, 1,
                        ph, xg, x.buf.C, x.H, x.W, osy=lay.stride, osx=lay.stride, ory=ph["ry"], orx=ph["rx"],
                        res=res, res_ld=res_ld, z=z, z_ld=z_ld, dact=dact, beta=beta)
                    npx = nb * ph["oh"] * ph["ow"]
                    frac = npx / float(nb * x.H * x.W)
                    o.meta = dict(cls="conv_dgrad",
                                  name=lay.name + (f" [phase {ph['ry']}{ph['rx']}]" if len(phases) > 1 else ""),
                                  flops=2.0 * npx * lay.cin * lay.cout * ph["th"] * ph["tw"],
                                  bytes=float(self.es * (frac * nb * out.H * out.W * lay.cout
                                                         + npx * lay.cin * (1 + (res is not None) + (z is not None) + beta)
                                                         + lay.cout * lay.cin * ph["th"] * ph["tw"])))
                    ops.append(o)
                return ops

            self._contrib(x, em)

    def _wgrad_s2_eligible(self, lay, x, out):
        """stride-2 3x3 pad-1 weight gradient as its four input phases on the halo kernel
        (include/dvie.h dvie_wgrad_desc.ws_taps; DVIE_WGRAD_S2=0 keeps the per-tap kernel,
        DVIE_WGRAD_S2=2 takes every eligible layer).  Default: inputs of >= 256 channels
        (transition1.1: 0.377 -> 0.297 ms/step); each phase launch streams the whole output
        gradient, so on the 64- / 128-channel inputs the four launches measured 2-35% slower
        than the per-tap kernel (profiles/r06e/)"""
        mode = os.environ.get("DVIE_WGRAD_S2", "1")
        if mode == "1" and x.c < 256:
            return False
        return (self.dtype == torch.bfloat16 and mode != "0" and lay.stride == 2
                and lay.kh == 3 and lay.kw == 3 and lay.pad == 1 and lay.dil == 1 and not lay.transposed
                and x.H % 2 == 0 and x.W % 2 == 0 and out.H == x.H // 2 and out.W == x.W // 2 and out.W % 64 == 0
                and x.c % 8 == 0 and x.buf.C % 8 == 0)

    def _emit_wgrad_s2(self, op, gout, gld):
        """The stride-2 weight gradient as four stride-1 launches, one per input phase
        (a, b): tap (i, j) of phase (a, b) is forward tap (kh, kw) = (1, .) for a = 0, (0 | 2, .)
        for a = 1 (i = 0 | 1; likewise for columns), read from the phase view x[2r + a][2q + b]
        (x + (a W + b) ld, x_ld 2 ld, iw = W as the row pitch); each launch fills its taps'
        column blocks of one [splits][cout][9 c] slab set, reduced once."""
        lay, x, out = op.layer, op.x, op.out
        nb = self.nb
        npix = nb * out.H * out.W
        lib = L.load()
        ops, slabs, bslabs = [], None, 0
        for a in (0, 1):
            for b in (0, 1):
                o = self._op(L.OP_WGRAD)
                d = o.u.wgrad
                d.g, d.x, d.ws = gout, self.ptr(x) + (a * x.W + b) * x.buf.C * self.es, 0
                d.g_ld, d.x_ld = gld, 2 * x.buf.C
                d.n, d.oh, d.ow, d.cout = nb, out.H, out.W, lay.cout_p
                d.ih, d.iw, d.c, d.sy, d.sx = x.H // 2, x.W, x.c, 1, 1
                d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = 1 + a, 1 + b, -a, -b, 1, 1
                khs, kws = ([1] if a == 0 else [0, 2]), ([1] if b == 0 else [0, 2])
                d.tmap = sum((kh * 3 + kw) << (4 * (i * len(kws) + j)) for i, kh in enumerate(khs)
                             for j, kw in enumerate(kws))
                d.ws_taps = 9
                d.dtype = self.dt
                hint = lib.dvie_wgrad_splits_hint(ctypes.byref(d))
                assert hint > 0, f"{lay.name}: the halo weight-gradient kernel refused a stride-2 phase launch"
                d.splits = hint
                n_s = lib.dvie_wgrad_slabs(ctypes.byref(d))
                assert slabs in (None, n_s), "stride-2 phase launches disagree on their slab count"
                slabs = n_s
                if a == 0 and b == 0 and lay.has_bias:  # the bias column sums ride on one launch
                    d.bws = 1
                    bslabs = lib.dvie_wgrad_bias_slabs(ctypes.byref(d))
                    d.bws = None
                    o.bws_off = slabs * lay.cout_p * 9 * x.c
                nt = len(khs) * len(kws)
                o.meta = dict(cls="conv_wgrad", name=lay.name + f" [phase {a}{b}]",
                              flops=2.0 * npix * lay.cout * lay.cin * nt,
                              bytes=float(self.es * (npix * lay.cout + npix * lay.cin)
                                          + 4 * slabs * lay.cout_p * nt * x.c))
                ops.append(o)
        wfl = slabs * lay.cout_p * 9 * x.c
        self.ws_floats = max(self.ws_floats, wfl + bslabs * lay.cout_p)
        self.bwd += ops
        self._emit_wreduce(lay, slabs, 9 * x.c, x.c, bslabs, wfl)

    def _emit_wreduce(self, lay, slabs, ws_k, c, bslabs, bias_off):
        """the slab reductions of a weight gradient (and of its bias partials) into the .grad
        views, and the layer's completion bookkeeping"""
        o = self._op(L.OP_WREDUCE)
        r = o.u.wreduce
        r.ws, r.dw, r.cmap = 0, 0, lay.cmap_t.data_ptr()
        r.splits, r.ws_rows, r.ws_k, r.co_off = slabs, lay.cout_p, ws_k, 0
        r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, lay.cin, lay.kh, lay.kw, c
        first = lay not in self.wg_first
        r.beta = 0 if first else 1
        o.meta = _reduce_meta(lay.name, r)
        self.bwd.append(o)
        self._grad_slots.append((len(self.bwd) - 1, lay, "weight", first))
        if lay.has_bias:
            o = self._op(L.OP_WREDUCE)
            r = o.u.wreduce
            r.ws, r.dw, r.cmap = 0, 0, None
            r.splits, r.ws_rows, r.ws_k, r.co_off = bslabs, lay.cout_p, 1, 0
            r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, 1, 1, 1, 1
            r.beta = 0 if first else 1
            o.meta = _reduce_meta(lay.name + ".bias", r)
            o.ws_off = bias_off
            self.bwd.append(o)
            self._grad_slots.append((len(self.bwd) - 1, lay, "bias", first))
        self.wg_first[lay] = True
        self._uses_left[lay] -= 1
        if self._uses_left[lay] == 0:
            self.completions.append((len(self.bwd), lay))

    def _emit_wgrad(self, op, gout, gld):
        """weight (and bias) gradient of a conv: split-K partial slabs + reduction into the
        OIHW .grad view, appended to the backward list (weight lane)."""
        lay, x, out = op.layer, op.x, op.out
        if self._wgrad_s2_eligible(lay, x, out) and gld % 8 == 0:
            return self._emit_wgrad_s2(op, gout, gld)
        nb = self.nb
        npix = nb * out.H * out.W
        taps = lay.fwd_taps()
        # weight gradient: split-K partial slabs + reduction into the OIHW .grad view
        tiles = rup(lay.cout_p, 64) // 64 * (rup(x.c, 64) // 64)
        ntap = lay.kh * lay.kw
        bkp = 64 if self.dtype == torch.bfloat16 else 32
        splits = max(1, min(max(1, npix // (bkp * 4)), 1024 // max(1, tiles * ntap)))
        o = self._op(L.OP_WGRAD)
        d = o.u.wgrad
        d.g, d.x, d.ws = gout, self.ptr(x), 0
        d.g_ld, d.x_ld = gld, x.buf.C
        d.n, d.oh, d.ow, d.cout = nb, out.H, out.W, lay.cout_p
        d.ih, d.iw, d.c, d.sy, d.sx = x.H, x.W, x.c, lay.stride, lay.stride
        d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = taps["th"], taps["tw"], taps["dy0"], taps["dx0"], taps["ddy"], \
            taps["ddx"]
        d.dtype = self.dt
        lib = L.load()
        hint = lib.dvie_wgrad_splits_hint(ctypes.byref(d))  # the halo kernel's preferred split
        d.splits = hint if hint > 0 else splits
        slabs = lib.dvie_wgrad_slabs(ctypes.byref(d))
        wfl = slabs * lay.cout_p * ntap * x.c
        bslabs = 0
        if lay.has_bias:  # bias column sums ride on the weight-gradient launch (d.bws)
            d.bws = 1  # placeholder (set in _finalize): makes the query see a bias launch
            bslabs = lib.dvie_wgrad_bias_slabs(ctypes.byref(d))
            d.bws = None
            o.bws_off = wfl
        self.ws_floats = max(self.ws_floats, wfl + bslabs * lay.cout_p)
        o.meta = dict(cls="conv_wgrad", name=lay.name, flops=2.0 * npix * lay.cout * lay.cin * ntap,
                      bytes=float(self.es * (npix * lay.cout + nb * x.H * x.W * lay.cin)
                                  + 4 * slabs * lay.cout_p * ntap * x.c))
        self.bwd.append(o)
        o = self._op(L.OP_WREDUCE)
        r = o.u.wreduce
        r.ws, r.dw, r.cmap = 0, 0, lay.cmap_t.data_ptr()
        r.splits, r.ws_rows, r.ws_k, r.co_off = slabs, lay.cout_p, ntap * x.c, 0
        r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, lay.cin, lay.kh, lay.kw, x.c
        first = lay not in self.wg_first
        r.beta = 0 if first else 1
        o.meta = _reduce_meta(lay.name, r)
        self.bwd.append(o)
        self._grad_slots.append((len(self.bwd) - 1, lay, "weight", first))
        if lay.has_bias:
            o = self._op(L.OP_WREDUCE)
            r = o.u.wreduce
            r.ws, r.dw, r.cmap = 0, 0, None
            r.splits, r.ws_rows, r.ws_k, r.co_off = bslabs, lay.cout_p, 1, 0
            r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, 1, 1, 1, 1
            r.beta = 0 if first else 1
            o.meta = _reduce_meta(lay.name + ".bias", r)
            o.ws_off = wfl
            self.bwd.append(o)
            self._grad_slots.append((len(self.bwd) - 1, lay, "bias", first))
        self.wg_first[lay] = True
        self._uses_left[lay] -= 1
        if self._uses_left[lay] == 0:
            self.completions.append((len(self.bwd), lay))

    def _im2col_dgrad(self, lay, x, phases):
        """Narrow-input stride-1 data gradients (HRNet's 3x3 448->3 / 448->20 heads: the
        output gradient has 8 / 24 channels) run as im2col + 1x1 GEMM over K = 9*c (128 /
        256) instead of the halo kernel's 9 taps x 64 padded channels (bf16 only).  Opt-in
        (DVIE_IM2COL_DGRAD=1): measured at 8x256x512 the 448->3 head goes 0.838 -> 0.756 ms
        but the 448->20 head 0.847 -> 0.942 ms (im2col 0.16 ms + GEMM 0.78 ms), no net gain:
        the GEMM's 448-channel output + activation-derivative read, not the padded MFMA work,
        bound these layers."""
        if self.dtype != torch.bfloat16 or os.environ.get("DVIE_IM2COL_DGRAD", "0") != "1":
            return False
        if lay.stride != 1 or len(phases) != 1:
            return False
        ph, _, kpad = phases[0]
        return (ph["th"] * ph["tw"] > 1 and lay.cout_p % 8 == 0 and lay.cout_p <= 32 and x.c >= 128
                and kpad % 64 == 0 and ph["ry"] == 0 and ph["rx"] == 0)

    def _im2col_dgrad_ops(self, lay, x, xg, out, gout, gld, phase, res, res_ld, z, z_ld, dact, beta):
        ph, wt, kpad = phase
        nb = self.nb
        npx = nb * ph["oh"] * ph["ow"]
        # one scratch shared by the layers (in order on the data lane)
        buf = self.__dict__.get("_i2c")
        if buf is None or buf.numel() < npx * kpad:
            buf = torch.empty(npx * kpad, dtype=self.dtype, device=self.device)
            self._i2c = buf
            self.keep.append(buf)
        e = self.ew_desc(L.EW_IM2COL, nb, out.H, out.W, kpad, buf.data_ptr(), kpad,
                         srcs=[(gout, gld, ph["th"], ph["tw"]), (None, 0, ph["dy0"], ph["dx0"]),
                               (None, 0, ph["ddy"], ph["ddx"])])
        e.u.ew.nsrc, e.u.ew.ext_c = 1, lay.cout_p
        e.meta = dict(cls="pointwise", name=lay.name + ".im2col", flops=0.0,
                      bytes=float(self.es * npx * (lay.cout_p + kpad)))
        one = dict(th=1, tw=1, dy0=0, dx0=0, ddy=1, ddx=1)
        o = self.conv_desc(buf.data_ptr(), kpad, nb, out.H, out.W, kpad, wt.data_ptr(), kpad, x.c, ph["oh"], ph["ow"],
                           1, 1, one, xg, x.buf.C, x.H, x.W, res=res, res_ld=res_ld, z=z, z_ld=z_ld, dact=dact,
                           beta=beta)
        o.meta = dict(cls="conv_dgrad", name=lay.name, flops=2.0 * npx * lay.cin * lay.cout * ph["th"] * ph["tw"],
                      bytes=float(self.es * (npx * kpad + npx * lay.cin * (1 + (res is not None) + (z is not None)
                                                                            + beta) + lay.cout * lay.cin * 9)))
        return [e, o]

    def _convT_backward(self, op, gout, gld):
        """nn.ConvTranspose2d backward through its virtual conv (see ConvLayer): the input
        gradient is that conv run forward over the ConvT output gradient; the weight gradient
        is that conv's weight gradient with its 'input' = the ConvT output gradient and its
        'output gradient' = the ConvT input activation; the bias gradient is the column sums
        of the ConvT output gradient."""
        lay, x, out = op.layer, op.x, op.out
        nb = self.nb
        taps = lay.fwd_taps()
        ntap = lay.kh * lay.kw
        if lay.trainable:
            npix = nb * x.H * x.W
            tiles = rup(lay.cout_p, 64) // 64 * (rup(out.c, 64) // 64)
            bkp = 64 if self.dtype == torch.bfloat16 else 32
            splits = max(1, min(max(1, npix // (bkp * 4)), 1024 // max(1, tiles * ntap)))
            o = self._op(L.OP_WGRAD)
            d = o.u.wgrad
            d.g, d.x, d.ws = self.ptr(x), gout, 0
            d.g_ld, d.x_ld = x.buf.C, gld
            d.n, d.oh, d.ow, d.cout = nb, x.H, x.W, lay.cout_p
            d.ih, d.iw, d.c, d.sy, d.sx = out.H, out.W, out.c, lay.stride, lay.stride
            d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = taps["th"], taps["tw"], taps["dy0"], taps["dx0"], 1, 1
            d.dtype = self.dt
            lib = L.load()
            hint = lib.dvie_wgrad_splits_hint(ctypes.byref(d))
            d.splits = hint if hint > 0 else splits
            slabs = lib.dvie_wgrad_slabs(ctypes.byref(d))
            self.ws_floats = max(self.ws_floats, slabs * lay.cout_p * ntap * out.c)
            o.meta = dict(cls="conv_wgrad", name=lay.name, flops=2.0 * npix * lay.cout * lay.cin * ntap,
                          bytes=float(self.es * (npix * lay.cout + nb * out.H * out.W * lay.cin)))
            self.bwd.append(o)
            o = self._op(L.OP_WREDUCE)
            r = o.u.wreduce
            r.ws, r.dw, r.cmap = 0, 0, lay.cmap_t.data_ptr()
            r.splits, r.ws_rows, r.ws_k, r.co_off = slabs, lay.cout_p, ntap * out.c, 0
            r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cout, lay.cin, lay.kh, lay.kw, out.c
            first = lay not in self.wg_first
            r.beta = 0 if first else 1
            self.bwd.append(o)
            self._grad_slots.append((len(self.bwd) - 1, lay, "weight", first))
            if lay.has_bias:
                opix = nb * out.H * out.W
                csplits = max(1, min(2048, opix // 512))
                o = self._op(L.OP_COLSUM)
                cd = o.u.colsum
                cd.g, cd.ws, cd.g_ld, cd.rows, cd.c, cd.splits, cd.dtype = gout, 0, gld, opix, out.c, csplits, self.dt
                self.ws_floats = max(self.ws_floats, csplits * out.c)
                self.bwd.append(o)
                o = self._op(L.OP_WREDUCE)
                r = o.u.wreduce
                r.ws, r.dw, r.cmap = 0, 0, None
                r.splits, r.ws_rows, r.ws_k, r.co_off = csplits, out.c, 1, 0
                r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c = lay.cin, 1, 1, 1, 1
                r.beta = 0 if first else 1
                self.bwd.append(o)
                self._grad_slots.append((len(self.bwd) - 1, lay, "bias", first))
            self.wg_first[lay] = True
            self._uses_left[lay] -= 1
            if self._uses_left[lay] == 0:
                self.completions.append((len(self.bwd), lay))
        if x.buf.needs_grad:
            xg = self.ptr(x, grad=True)

            def em(beta, res, res_ld, dact, z, z_ld, lay=lay, x=x, xg=xg, out=out, gout=gout, gld=gld):
                o = self.conv_desc(gout, gld, nb, out.H, out.W, out.c, lay.wf.data_ptr(), lay.kpad, lay.cout_p,
                                   x.H, x.W, lay.stride, lay.stride, taps, xg, x.buf.C, x.H, x.W,
                                   res=res, res_ld=res_ld, z=z, z_ld=z_ld, dact=dact, beta=beta)
                npx = nb * x.H * x.W
                o.meta = dict(cls="conv_dgrad", name=lay.name, flops=2.0 * npx * lay.cout * lay.cin * ntap,
                              bytes=float(self.es * (nb * out.H * out.W * lay.cin + npx * lay.cout)))
                return [o]

            self._contrib(x, em)

    # ---------------- finalize ----------------
    def _batch_reductions(self):
        """The weight lane's slab reductions in batches of up to 16, each batch ONE
        dvie_wgrad_reduce_multi launch where its last reduction was (include/dvie.h).  Without
        batching every slab writer (weight gradient / column sums) shares offset 0 of self.ws,
        each reduced right after it is written; in a batch each writer gets its own region
        (consecutive writers with no reduction between them -- the stride-2 phase launches of
        one slab set -- share one), so the reductions can wait for the batch's end.  Measured
        with the timing-only skip (tools/skip_ab.sh): the 73 one-by-one reductions cost the eager
        step 0.8 ms of its 31.3.  DVIE_WREDUCE_MULTI=0 keeps them one by one."""
        if os.environ.get("DVIE_WREDUCE_MULTI", "1") == "0" or not self.bwd:
            return
        MAXN = 16
        budget = int(float(os.environ.get("DVIE_WREDUCE_MB", "1024")) * 2 ** 20 / 4)  # floats per batch
        # pass 1: reductions reading self.ws -> their writer; region sizes per writer group
        writer_of, size, cur, had_reduce = {}, {}, None, True
        for i, o in enumerate(self.bwd):
            if o.kind in (L.OP_WGRAD, L.OP_COLSUM):
                if had_reduce or cur is None:
                    cur, had_reduce = i, False
                writer_of[i] = cur
            elif o.kind == L.OP_WREDUCE:
                had_reduce = True
                if getattr(o, "ws_ptr", None) is None:
                    r = o.u.wreduce
                    writer_of[i] = cur
                    size[cur] = max(size.get(cur, 0), getattr(o, "ws_off", 0) + r.splits * r.ws_rows * r.ws_k)
        # pass 2: batches, regions, the multi ops
        new, remap, pending, base, off, live_end = [], {}, [], {}, 0, 0
        self._multi = []  # (host descriptor array, [(ws_ptr or None, float offset in self.ws)])

        def flush():
            nonlocal pending, off
            if not pending:
                return
            arr = (L.WreduceDesc * len(pending))()
            wsrc = []
            for j, (oi, o) in enumerate(pending):
                arr[j] = o.u.wreduce
                wp = getattr(o, "ws_ptr", None)
                wsrc.append((wp, None if wp else base[writer_of[oi]] + getattr(o, "ws_off", 0)))
            m = self._op(L.OP_WREDUCE_MULTI)
            m.u.wreduce_multi.descs = ctypes.addressof(arr)
            m.u.wreduce_multi.n = len(pending)
            metas = [getattr(o, "meta", None) or {} for _, o in pending]
            m.meta = dict(cls="wgrad_reduce", name=f"{len(pending)} reductions ({metas[0].get('name', '')} ..)",
                          flops=0.0, bytes=float(sum(mt.get("bytes", 0.0) for mt in metas)))
            self._multi.append((arr, wsrc))
            for oi, _ in pending:
                remap[oi] = len(new)
            new.append(m)
            pending, off = [], 0

        # a batch's reductions run concurrently: two that accumulate into one gradient (a layer
        # used twice, e.g. the seg encoder on both segmentation maps) go to different batches
        target = {idx: (id(lay), which) for idx, lay, which, _ in self._grad_slots if which != "bn"}
        for i, o in enumerate(self.bwd):
            if o.kind == L.OP_WREDUCE and i in target and any(target.get(oi) == target[i] for oi, _ in pending):
                flush()
                off = live_end  # the latest region may still be read: the next ones go after it
            if o.kind in (L.OP_WGRAD, L.OP_COLSUM):
                w = writer_of[i]
                if w == i:  # a new slab region
                    need = size.get(w, 0)
                    if pending and off + need > budget:
                        flush()  # (every earlier region has all its reductions in that batch)
                    base[w] = off
                    off += need
                    live_end = off
                self.ws_floats = max(self.ws_floats, base[w] + size.get(w, 0))
                o.ws_base = base[w]
                remap[i] = len(new)
                new.append(o)
            elif o.kind == L.OP_WREDUCE:
                pending.append((i, o))
                if len(pending) == MAXN:
                    flush()
                    off = live_end  # (the latest region's other reductions may follow)
            else:
                remap[i] = len(new)
                new.append(o)
        flush()
        self.bwd = new
        self.completions = [(remap[idx - 1] + 1, lay) for idx, lay in self.completions]
        # backward indices recorded while building: moved with their ops
        self.ext_ograd = {k: remap[i] for k, i in self.ext_ograd.items()}
        if hasattr(self, "ext_head_grad"):
            self.ext_head_grad = {k: remap[i] for k, i in self.ext_head_grad.items()}
        self.ext_grad = {k: [(remap[i], op) for i, op in v] for k, v in self.ext_grad.items()}
        if hasattr(self, "ext_mask"):
            self.ext_mask = {k: [(w, remap[i] if w == "bwd" else i, op) for w, i, op in v]
                             for k, v in self.ext_mask.items()}
        slots = []
        pos = {}  # multi op index -> the old indices of its reductions, in order
        for oi, ni in sorted(remap.items()):
            if new[ni].kind == L.OP_WREDUCE_MULTI:
                pos.setdefault(ni, []).append(oi)
        for idx, lay, which, first in self._grad_slots:
            if which != "bn" and self.bwd[remap[idx]].kind == L.OP_WREDUCE_MULTI:
                ni = remap[idx]
                slots.append((("multi", ni, pos[ni].index(idx)), lay, which, first))
            else:
                slots.append((remap[idx], lay, which, first))
        self._grad_slots = slots
        self.n_bwd = len(self.bwd)

    def _wreduce_desc(self, idx):
        """the dvie_wreduce_desc of a gradient slot (one reduction op, or an element of a
        batch's host array)"""
        if isinstance(idx, tuple):
            _, ni, j = idx
            arr = (L.WreduceDesc * self.bwd_arr[ni].u.wreduce_multi.n).from_address(
                self.bwd_arr[ni].u.wreduce_multi.descs)
            return arr[j]
        return self.bwd_arr[idx].u.wreduce

    def _finalize(self):
        L.load()
        self._batch_reductions()
        # workspace for wgrad / colsum partials
        self.ws = torch.empty(max(1, self.ws_floats), dtype=torch.float32, device=self.device)
        self.keep.append(self.ws)
        wlane = _wgrad_lane()
        wsp = self.ws.data_ptr()
        for o in self.bwd:
            # weight / bias gradients are off the data-gradient chain: they run on the
            # executor's side stream (dvie_op.lane 1), forked where their output gradient is
            # final and joined at the end of each dvie_run_ops call.  They are the only users
            # of self.ws, and they stay in order on that one stream.
            if o.kind in (L.OP_WGRAD, L.OP_WREDUCE, L.OP_COLSUM, L.OP_WREDUCE_MULTI) and wlane:
                o.lane = 1
            if o.kind == L.OP_WGRAD:
                o.u.wgrad.ws = wsp + 4 * getattr(o, "ws_base", 0)
                if hasattr(o, "bws_off"):  # bias partials after the weight slabs
                    o.u.wgrad.bws = wsp + 4 * (getattr(o, "ws_base", 0) + o.bws_off)
            elif o.kind == L.OP_COLSUM:
                o.u.colsum.ws = wsp + 4 * getattr(o, "ws_base", 0)
            elif o.kind == L.OP_WREDUCE:
                o.u.wreduce.ws = getattr(o, "ws_ptr", None) or wsp + 4 * getattr(o, "ws_off", 0)
        for arr, wsrc in getattr(self, "_multi", []):
            for j, (wp, off) in enumerate(wsrc):
                arr[j].ws = wp if wp else wsp + 4 * off
            self.keep.append(arr)
        # pack op (all layers, one launch) goes first in the forward list
        descs = self._pack_descs
        if not descs:  # no convolutions (e.g. a pointwise-only plan)
            self.fwd_arr = (L.Op * max(1, len(self.fwd)))(*self.fwd)
            self.fwd_off = 0
            self.bwd_arr = (L.Op * max(1, len(self.bwd)))(*self.bwd) if self.bwd else None
            self.n_bwd = len(self.bwd)
            return
        blk = 0  # flat grid: each descriptor's first block (csrc/conv.hip pack_kernel)
        for d in descs:
            d.blk0 = blk
            blk += pack_blocks(d)
        arr = (L.PackDesc * len(descs))(*descs)
        raw = bytes(arr)
        dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self.keep.append(dev)
        po = self._op(L.OP_PACK)
        po.u.pack.descs_dev = dev.data_ptr()
        po.u.pack.n = len(descs)
        po.u.pack.blocks = blk
        self.fwd_arr = (L.Op * (len(self.fwd) + 1))(po, *self.fwd)
        self.fwd_off = 1
        self.bwd_arr = (L.Op * max(1, len(self.bwd)))(*self.bwd) if self.bwd else None
        self.n_bwd = len(self.bwd)

    # ---------------- execution ----------------
    def set_input(self, key, t):
        """Patch the external NCHW fp32 input `t` (any strides) into the forward list."""
        assert t.dtype == torch.float32 and t.device.type == self.device.type
        for idx, op in self.ext_in[key]:
            d = self.fwd_arr[idx + self.fwd_off].u.ew
            assert t.shape[0] == self._part(op.part)[1], (key, tuple(t.shape), self.nf)
            assert t.shape[2:] == (op.out.H, op.out.W) and t.shape[1] >= op.ext_c0 + op.ext_c, (key, tuple(t.shape))
            sn, sc, sh, sw = t.stride()
            d.ext = t.data_ptr() + 4 * op.ext_c0 * sc
            d.sn, d.sc, d.sh, d.sw = sn, sc, sh, sw
            d.src1, d.sh1 = None, 0

    def set_input_parts(self, key, parts):
        """set_input for an input given as consecutive channel blocks (the frames of a clip
        as separate NCHW fp32 tensors of equal shape and strides) instead of one concatenated
        tensor: each input op reads its channels in place; an op whose channels straddle two
        blocks reads the second through the EW_NCHW split (src1 / sh1)."""
        starts = [0]
        for t in parts:
            assert t.dtype == torch.float32 and t.device.type == self.device.type
            assert t.stride() == parts[0].stride() and t.shape[0] == parts[0].shape[0], (key, t.shape, t.stride())
            starts.append(starts[-1] + t.shape[1])
        for idx, op in self.ext_in[key]:
            d = self.fwd_arr[idx + self.fwd_off].u.ew
            j = max(i for i in range(len(parts)) if starts[i] <= op.ext_c0)
            t = parts[j]
            assert t.shape[0] == self._part(op.part)[1] and t.shape[2:] == (op.out.H, op.out.W), (key, tuple(t.shape))
            sn, sc, sh, sw = t.stride()
            d.ext = t.data_ptr() + 4 * (op.ext_c0 - starts[j]) * sc
            d.sn, d.sc, d.sh, d.sw = sn, sc, sh, sw
            end = op.ext_c0 + op.ext_c
            if end > starts[j + 1]:  # the op's channels continue in the next block
                assert j + 1 < len(parts) and end <= starts[j + 2], (key, op.ext_c0, op.ext_c, starts)
                d.src1, d.sh1 = parts[j + 1].data_ptr(), starts[j + 1] - op.ext_c0
            else:
                d.src1, d.sh1 = None, 0

    def set_output(self, name, t):
        for idx, region in self.ext_out[name]:
            d = self.fwd_arr[idx + self.fwd_off].u.conv
            d.y = t.data_ptr() + region.c0 * t.element_size()
            d.y_ld = t.shape[-1]

    def set_mask(self, key, t):
        """Patch the external NCHW fp32 mask `key` (channel op.chan of t) into its ops."""
        assert t.dtype == torch.float32 and t.device.type == self.device.type
        sn, sc, sh, sw = t.stride()
        for where, idx, op in getattr(self, "ext_mask", {}).get(key, []):
            d = (self.fwd_arr[idx + self.fwd_off] if where == "fwd" else self.bwd_arr[idx]).u.ew
            d.ext = t.data_ptr() + 4 * op.chan * sc
            d.sn, d.sc, d.sh, d.sw = sn, sc, sh, sw

    def set_output_nchw(self, key, t):
        """Point the NCHW sink `key` at an fp32 tensor (any strides)."""
        assert t.dtype == torch.float32
        d = self.fwd_arr[self.ext_nchw_out[key] + self.fwd_off].u.ew
        sn, sc, sh, sw = t.stride()
        d.ext = t.data_ptr()
        d.sn, d.sc, d.sh, d.sw = sn, sc, sh, sw

    def set_head_output(self, key, t):
        """Point head `key` at an fp32 vector of length n*(h/pool)*(w/pool)."""
        idx, rows = self.ext_head[key]
        assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == rows
        self.fwd_arr[idx + self.fwd_off].u.head.out = t.data_ptr()

    def set_head_grad(self, key, t):
        t = t.contiguous()
        assert t.dtype == torch.float32
        self.bwd_arr[self.ext_head_grad[key]].u.head.gout = t.data_ptr()
        self.keep_grad = t

    def set_output_grad(self, key, t):
        """Patch the incoming gradient (fp32, any strides, logical NCHW) of output `key`."""
        assert t.dtype == torch.float32
        d = self.bwd_arr[self.ext_ograd[key]].u.ew
        sn, sc, sh, sw = t.stride()
        d.ext = t.data_ptr()
        d.sn, d.sc, d.sh, d.sw = sn, sc, sh, sw

    def set_l1_loss(self, out=None, value_scale=1.0, grad_scale=1.0):
        """Where the VGG feature-L1 loss ops put their values, and the gradient scale.
        out None: level k's mean into l1_out[k] (the autograd path, VGGLoss); a 1-element
        fp32 tensor: value_scale * (mean over levels of the level means) into out[0] (the
        levels add into it in order, no PyTorch reduction).  grad_scale multiplies the
        backward seeds, so the input gradient is grad_scale * d(loss)/d(pred)."""
        nl = max(1, len(self._l1_fwd))
        for k, (idx, lev) in enumerate(self._l1_fwd):
            d = self.fwd_arr[idx + self.fwd_off].u.loss
            if out is None:
                d.out, d.out_acc, d.out_scale = self.l1_out.data_ptr() + 4 * lev, 0, 1.0
            else:
                d.out, d.out_acc, d.out_scale = out.data_ptr(), int(k > 0), value_scale / nl
        if self.bwd_arr is not None:
            if not hasattr(self, "_l1_bwd"):
                self._l1_bwd = [(i, o.l1_seed) for i, o in enumerate(self.bwd) if hasattr(o, "l1_seed")]
            for i, base in self._l1_bwd:
                self.bwd_arr[i].u.ew.scale = base * grad_scale

    def set_input_grad(self, key, t, accumulate=False):
        for idx, op in self.ext_grad[key]:
            d = self.bwd_arr[idx].u.ew
            sn, sc, sh, sw = t.stride()
            d.ext = t.data_ptr() + 4 * op.ext_c0 * sc
            d.sn, d.sc, d.sh, d.sw = sn, sc, sh, sw
            d.beta = int(accumulate)

    def set_param_grads(self, accumulate=False, fresh=()):
        """Point weight reductions at the parameters' .grad tensors (fp32, OIHW).  `fresh`:
        ids of conv modules whose weight gradient this backward overwrites whatever
        `accumulate` says (SpectralNorm's per-call d(W_bar / sigma) scratch)."""
        for idx, lay, which, first in self._grad_slots:
            if which == "bn":  # lay is the BatchNorm module: gamma and beta gradients
                d = self.bwd_arr[idx].u.bn
                for pname, field in (("weight", "dgamma"), ("bias", "dbeta")):
                    p = getattr(lay, pname)
                    if p is None:
                        continue
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                    setattr(d, field, p.grad.data_ptr())
                d.accumulate = int(accumulate) if first else 1
                continue
            d = self._wreduce_desc(idx)
            if isinstance(lay.m, StackedConv):
                d.dw = lay.m.grad_ptr(which)
            else:
                p = getattr(lay.m, which)
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                d.dw = p.grad.data_ptr()
            if first:
                d.beta = 0 if (which == "weight" and id(lay.m) in fresh) else int(accumulate)

    def activation_signs(self):
        """{buffer name: bool NCHW CPU tensor (value > 0)} for every buffer written by a
        LeakyReLU- or ReLU-activated op in the last forward (test support: which branch each
        activation took, so an fp64 oracle can be evaluated on the same branches).  A buffer
        with other producers too (the HRNet concat) is included whole; the caller reads the
        channel slice its activated producer wrote."""
        out = {}
        for b in self.g.buffers:
            if b.t is not None and any(p.act in (L.ACT_LRELU, L.ACT_RELU) for p in b.producers):
                out[b.name] = (b.t > 0).permute(0, 3, 1, 2).cpu()
        return out

    def activation_list(self):
        """[bool NCHW CPU tensor (value > 0) of the output region of every LeakyReLU- or
        ReLU-activated op, in forward op order] for the last forward (test support: an
        oracle that applies its activations in the same order consumes them one by one;
        padded channels included, the caller slices the real ones)."""
        out = []
        for op in self.g.ops:
            r = getattr(op, "out", None)
            if r is None or getattr(op, "act", 0) not in (L.ACT_LRELU, L.ACT_RELU) or r.buf.t is None:
                continue
            out.append((r.buf.t[..., r.c0:r.c0 + r.c] > 0).permute(0, 3, 1, 2).cpu())
        return out

    def _nonfinite(self):
        """names of buffers (activations / gradients) holding non-finite values (debug)."""
        out = set()
        for b in self.g.buffers:
            for tag, t in (("A", b.t), ("G", b.g)):
                if t is not None and t.is_floating_point() and not bool(torch.isfinite(t).all()):
                    out.add(f"{tag}:{b.name}")
        return out

    def _run(self, arr, start, end, s, what, metas):
        lib = L.load()
        base = ctypes.addressof(arr)
        sz = ctypes.sizeof(L.Op)
        if DEBUG_NAN:  # op-by-op, report the first op after which new buffers turn non-finite
            seen = self._nonfinite()
            for i in range(start, end):
                L.check(lib.dvie_run_ops(base + i * sz, 1, s), what)
                torch.cuda.synchronize()
                now = self._nonfinite()
                if now - seen:
                    print(f"[dvie nan] {what} op {i} kind {arr[i].kind} meta {metas[i] if metas else None}: "
                          f"{sorted(now - seen)}", flush=True)
                    seen = now
            return
        if OP_HOOK is not None:  # op by op, each handed to the hook (which runs it)
            for i in range(start, end):
                OP_HOOK(self, arr, i, metas[i] if metas else None,
                        lambda i=i: L.check(lib.dvie_run_ops(base + i * sz, 1, s), what))
            return
        if PROFILE is None:
            L.check(lib.dvie_run_ops(base + start * sz, end - start, s), what)
            return
        for i in range(start, end):  # op-by-op with events (profiling steps only)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            lane, arr[i].lane = arr[i].lane, 0  # on the timed stream: no side-stream wait in the timing
            e0.record()
            L.check(lib.dvie_run_ops(base + i * sz, 1, s), what)
            e1.record()
            arr[i].lane = lane
            PROFILE.append((metas[i] if metas is not None else None, arr[i].kind, e0, e1))

    def invalidate_pack(self):
        """static_weights plans: repack at the next forward whatever the parameters' version
        counters say (a write through p.data bumps none)."""
        self._pack_sig = None

    def run_forward(self, stream=None):
        s = L.stream_ptr() if stream is None else stream
        metas = [None] * self.fwd_off + [getattr(o, "meta", None) for o in self.fwd]
        start = 0
        if self.fwd_off and self.static_weights:
            # frozen weights (VGG19, the loss network): pack once, again only when a source
            # tensor is replaced or modified in place (load_state_dict bumps its version)
            sig = tuple((t.data_ptr(), t._version) for t in self._pack_srcs)
            if sig == self._pack_sig:
                start = self.fwd_off
            self._pack_sig = sig
        self._run(self.fwd_arr, start, len(self.fwd_arr), s, "forward plan", metas)
        self.generation += 1

    def run_backward(self, stream=None, cuts=(), on_cut=None):
        """Run the backward list; with `cuts` (op indices), run it in segments and call
        on_cut(k) after segment k (used to launch gradient all-reduce buckets as soon as
        their parameters are final, overlapping communication with the rest)."""
        if self.n_bwd == 0:
            return
        s = L.stream_ptr() if stream is None else stream
        metas = [getattr(o, "meta", None) for o in self.bwd]
        start = 0
        for k, end in enumerate(list(cuts) + [self.n_bwd]):
            if end > start:
                self._run(self.bwd_arr, start, end, s, "backward plan", metas)
            start = max(start, end)
            if on_cut is not None and k < len(cuts):
                on_cut(k)

    def zero_grad_buffers(self):
        for b in self.g.buffers:
            if b.g is not None:
                b.g.zero_()

    def describe(self):
        kinds = {}
        for o in list(self.fwd) + list(self.bwd):
            kinds[o.kind] = kinds.get(o.kind, 0) + 1
        return dict(n_fwd=len(self.fwd) + 1, n_bwd=self.n_bwd, kinds=kinds, ws_mb=self.ws_floats * 4 / 2**20)


