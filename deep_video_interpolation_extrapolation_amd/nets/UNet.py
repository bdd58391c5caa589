"""UNet-family blocks (reference nets/UNet.py:16-157, nets/SepUNet.py:12-71,
nets/SubNets.py:14-29) on the MI355X plan engine.

Module trees, construction order (so seeded initialisation) and state_dict keys follow the
reference: double_conv / inconv / down / up / outconv, SegEncoder (the BatchNorm variant of
SubNets.py), UNet and SepUNet.  SepUNet lowers to one engine plan: HIP convs (bias
epilogue), BatchNorm with batch statistics fused with its LeakyReLU(0.2), bilinear x2
upsampling with align_corners=True written straight into the channel slices of the
decoder concat (up(cat(a, b, c)) = cat(up(a), up(b), up(c))), the fg/bg mask products
(nets/SepUNet.py:45-46), and the tanh RGB head.

Both networks are dormant in the reference (not selectable from options/options.py).
UNet as written cannot run: decoder_2 = up(256, 128) builds double_conv(256, ...) but is fed
cat(decon3, encon2) = 512 channels (nets/UNet.py:126,147), so its forward raises the same
channel-mismatch error here.  SepUNet's channel bookkeeping is consistent and it runs.
"""
import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import FlatParams, PlanFunction, PlanPool, precision_of
from .conv import Conv2d


class double_conv(nn.Module):
    """(conv => BN => LeakyReLU(0.2)) * 2   (nets/UNet.py:16-31)"""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Sequential(Conv2d(in_ch, out_ch, 3, padding=1), nn.BatchNorm2d(out_ch),
                                  nn.LeakyReLU(0.2, inplace=True),
                                  Conv2d(out_ch, out_ch, 3, padding=1), nn.BatchNorm2d(out_ch),
                                  nn.LeakyReLU(0.2, inplace=True))


class inconv(nn.Module):
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = double_conv(in_ch, out_ch)


class down(nn.Module):
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.mpconv = nn.Sequential(Conv2d(in_ch, out_ch, 3, stride=2, padding=1), nn.BatchNorm2d(out_ch),
                                    nn.LeakyReLU(0.2, inplace=True), double_conv(out_ch, out_ch))


class up(nn.Module):
    def __init__(self, in_ch, out_ch, bilinear=True):
        super().__init__()
        if not bilinear:
            raise NotImplementedError("up(bilinear=False) (ConvTranspose2d) is not used by the reference nets")
        self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self.conv = double_conv(in_ch, out_ch)


class outconv(nn.Module):
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = Conv2d(in_ch, out_ch, 1)


class SegEncoder(nn.Module):
    """nets/SubNets.py:14-29: conv-BN-LReLU, conv-BN-LReLU, conv (20 -> 4 channels)."""

    def __init__(self, in_dim, out_dim=4):
        super().__init__()
        self.in_dim, self.out_dim = in_dim, out_dim
        self.sequence = nn.Sequential(Conv2d(in_dim, 32, 3, 1, 1), nn.BatchNorm2d(32), nn.LeakyReLU(0.2, inplace=True),
                                      Conv2d(32, 32, 3, 1, 1), nn.BatchNorm2d(32), nn.LeakyReLU(0.2, inplace=True),
                                      Conv2d(32, out_dim, 3, 1, 1))


# ---------------- plan lowering helpers ----------------
def _cbr(g, x, conv, bn, name, trainable, cmap=None, out=None):
    """conv (+bias) -> BatchNorm (batch statistics) -> LeakyReLU(0.2), into `out` (a region)
    or a new buffer."""
    k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    hh, ww = (x.H + 2 * p - k) // s + 1, (x.W + 2 * p - k) // s + 1
    cp = E.rup(conv.out_channels, 8)
    t = g.buffer(name + ".pre", hh, ww, cp)
    g.conv(x, conv, E.R(t), cmap=cmap, trainable=trainable, name=name)
    if out is None:
        out = E.R(g.buffer(name, hh, ww, cp))
    g.bn(E.R(t), bn, out, act=L.ACT_LRELU, trainable=trainable)
    return out


def _double(g, x, dc, name, trainable, cmap=None):
    c = dc.conv
    h = _cbr(g, x, c[0], c[1], name + ".0", trainable, cmap=cmap)
    return _cbr(g, h, c[3], c[4], name + ".3", trainable)


def _down(g, x, d, name, trainable):
    m = d.mpconv
    h = _cbr(g, x, m[0], m[1], name + ".mpconv.0", trainable)
    return _double(g, h, m[3], name + ".mpconv.3.conv", trainable)


def _upcat(g, parts, name):
    """x2 bilinear (align_corners=True) upsample of cat(parts) into one buffer."""
    H, W = parts[0].H * 2, parts[0].W * 2
    c = sum(p.c for p in parts)
    u = g.buffer(name, H, W, c)
    off = 0
    for p in parts:
        g.fuse([p], E.R(u, off, p.c), align=True)
        off += p.c
    return E.R(u)


def _cat(g, parts, name):
    H, W = parts[0].H, parts[0].W
    c = sum(p.c for p in parts)
    u = g.buffer(name, H, W, c)
    off = 0
    for p in parts:
        g.fuse([p], E.R(u, off, p.c))
        off += p.c
    return E.R(u)


class SepUNet(FlatParams, nn.Module):
    """Reference nets/SepUNet.py:12-71.  forward(input, fg_mask, gt=None) -> (rgb, seg):
    input (B, 46, H, W) = [frames (6) | segs (40)], fg_mask (B, 2, H, W); H, W multiples
    of 8."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.in_channel = (3 + 4) * 2
        self.seg_encoder = SegEncoder(in_dim=20)
        self.fg_encoder_0 = inconv(self.in_channel, 32)
        self.fg_encoder_1 = down(32, 64)
        self.fg_encoder_2 = down(64, 128)
        self.fg_encoder_3 = down(128, 128)
        self.bg_encoder_0 = inconv(self.in_channel, 32)
        self.bg_encoder_1 = down(32, 64)
        self.bg_encoder_2 = down(64, 128)
        self.bg_encoder_3 = down(128, 128)
        self.decoder_3 = up(256, 256)
        self.decoder_2 = up(512, 128)
        self.decoder_1 = up(256, 64)
        self.decoder_0 = inconv(128, 32)
        self.rgb_decoder = Conv2d(32, 3, 3, padding=1)
        self.seg_decoder = Conv2d(32, 20, 3, padding=1)
        self.dtype = precision_of(args)
        self._pool = PlanPool(self._build_plan)
        self._flatten()

    def _lower(self, g, H, W, trainable):
        se = self.seg_encoder.sequence
        ins = {}
        for side in ("fg", "bg"):
            b = g.buffer(f"{side}_in", H, W, 16)  # [frames 6 (+2 zero) | seg-enc 0 (4) | seg-enc 1 (4)]
            g.input_nchw(E.R(b, 0, 8), "x", ext_c=6)
            ins[side] = b
        for k in range(2):
            s_in = g.buffer(f"seg{k}_in", H, W, 24)
            g.input_nchw(E.R(s_in), "seg", ext_c0=20 * k, ext_c=20)
            h = _cbr(g, E.R(s_in), se[0], se[1], f"seg_encoder.{k}.0", trainable)
            h = _cbr(g, h, se[3], se[4], f"seg_encoder.{k}.3", trainable)
            e = g.buffer(f"seg_encoder.{k}.6", H, W, 8)
            g.conv(h, se[6], E.R(e), trainable=trainable, name="seg_encoder.sequence.6")
            g.mask(E.R(e, 0, 4), E.R(ins["fg"], 8 + 4 * k, 4), "fg_mask", k, inverse=False)
            g.mask(E.R(e, 0, 4), E.R(ins["bg"], 8 + 4 * k, 4), "fg_mask", k, inverse=True)
        cmap = list(range(6)) + [-1, -1] + list(range(6, 14))
        enc = {}
        for side in ("fg", "bg"):
            e0 = _double(g, E.R(ins[side]), getattr(self, f"{side}_encoder_0").conv, f"{side}_encoder_0", trainable,
                         cmap=cmap)
            e1 = _down(g, e0, getattr(self, f"{side}_encoder_1"), f"{side}_encoder_1", trainable)
            e2 = _down(g, e1, getattr(self, f"{side}_encoder_2"), f"{side}_encoder_2", trainable)
            e3 = _down(g, e2, getattr(self, f"{side}_encoder_3"), f"{side}_encoder_3", trainable)
            enc[side] = (e0, e1, e2, e3)
        fg, bg = enc["fg"], enc["bg"]
        d3 = _double(g, _upcat(g, [fg[3], bg[3]], "decoder_3.up"), self.decoder_3.conv, "decoder_3", trainable)
        d2 = _double(g, _upcat(g, [d3, fg[2], bg[2]], "decoder_2.up"), self.decoder_2.conv, "decoder_2", trainable)
        d1 = _double(g, _upcat(g, [d2, fg[1], bg[1]], "decoder_1.up"), self.decoder_1.conv, "decoder_1", trainable)
        d0 = _double(g, _cat(g, [d1, fg[0], bg[0]], "decoder_0.cat"), self.decoder_0.conv, "decoder_0", trainable)
        rgb = g.buffer("rgb", H, W, 8)
        g.conv(d0, self.rgb_decoder, E.R(rgb), act=L.ACT_TANH, trainable=trainable, name="rgb_decoder")
        seg = g.buffer("seg", H, W, 24)
        g.conv(d0, self.seg_decoder, E.R(seg), trainable=trainable, name="seg_decoder")
        g.output_nchw("rgb", E.R(rgb), 3)
        g.output_nchw("seg", E.R(seg), 20)
        return g

    def _build_plan(self, key):
        n, H, W, dtype, bn_train, trainable, dev = key
        g = E.Graph(dtype)
        g.bn_training = bn_train
        self._lower(g, H, W, trainable)
        return g.compile(n, dev, backward=trainable)

    def _on_moved(self):
        self._pool.clear()

    def run_forward(self, inputs, train):
        x, seg, mask = inputs
        L.require_gpu(x)
        n, _, H, W = x.shape
        if H % 8 or W % 8:
            raise ValueError("SepUNet: H and W must be multiples of 8 (three stride-2 levels)")
        trainable = bool(train) and any(p.requires_grad for p in self.parameters())
        plan = self._pool.acquire((n, H, W, self.dtype, self.training, trainable, x.device))
        plan.set_input("x", x)
        plan.set_input("seg", seg)
        plan.set_mask("fg_mask", mask)
        rgb = torch.empty((n, 3, H, W), dtype=torch.float32, device=x.device)
        sg = torch.empty((n, 20, H, W), dtype=torch.float32, device=x.device)
        plan.set_output_nchw("rgb", rgb)
        plan.set_output_nchw("seg", sg)
        plan.run_forward()
        self.last_plan = plan
        if self.training:  # one increment per BatchNorm call, as nn.BatchNorm2d.train()
            for op in plan.g.ops:
                if isinstance(op, E.BNOp) and op.m.num_batches_tracked is not None:
                    op.m.num_batches_tracked.add_(1)
        return plan, (rgb, sg)

    def run_backward(self, plan, inputs, grads, needs):
        g_rgb, g_seg = grads
        plan.set_param_grads(self.grad_views())
        plan.set_output_grad("rgb", (g_rgb if g_rgb is not None else torch.zeros_like(inputs[0][:, :3])).float())
        plan.set_output_grad("seg", (g_seg if g_seg is not None else
                                     torch.zeros((inputs[0].shape[0], 20) + inputs[0].shape[2:],
                                                 device=inputs[0].device)).float())
        plan.run_backward()
        return [None, None, None]

    def forward(self, input, fg_mask=None, gt=None):
        if fg_mask is None:
            raise ValueError("SepUNet needs fg_mask (B, 2, H, W) (nets/SepUNet.py:45-46)")
        x = input[:, :6].float()
        seg = input[:, 6:46].float()
        return PlanFunction.apply(self, 3, x, seg, fg_mask.float().detach(), *self._flat_params)


class UNet(nn.Module):
    """Reference nets/UNet.py:109-157 (module tree only; see the module docstring)."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.in_channel = (3 + 4) * 2
        self.seg_encoder = SegEncoder(in_dim=20)
        self.encoder_0 = inconv(self.in_channel, 64)
        self.encoder_1 = down(64, 128)
        self.encoder_2 = down(128, 256)
        self.encoder_3 = down(256, 256)
        self.decoder_3 = up(256, 256)
        self.decoder_2 = up(256, 128)
        self.decoder_1 = up(128, 64)
        self.decoder_0 = inconv(64, 32)
        self.rgb_decoder = Conv2d(32, 3, 3, padding=1)
        self.seg_decoder = Conv2d(32, 20, 3, padding=1)

    def forward(self, input, fg_mask=None, gt=None):
        raise RuntimeError("UNet (reference nets/UNet.py:147): decoder_2 = up(256, 128) expects 256 input "
                           "channels but receives cat([decon3, encon2]) = 512 channels; the reference "
                           "network cannot run as written")
