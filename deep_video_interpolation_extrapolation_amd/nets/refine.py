"""Second-stage refinement nets on the MI355X plan engine.

  SRNRefine        reference nets/refine_nets.py:27-135
  MSResAttnRefine  reference nets/refine_nets.py:138-399

Module trees, construction order (hence seeded initialisation) and parameter names follow
the reference, so its checkpoints load unchanged.  Each net lowers to ONE engine plan
covering all n_scales scales (weights shared across scales, streams and uses):

* SRNRefine: per scale (coarsest first) the 40-channel input [rgb | previous prediction |
  seg | encoded features] is resized on the device (bilinear, align_corners=True); the
  previous prediction enters detached (refine_nets.py:111) while the hidden bottleneck
  state is carried to the next scale with its gradient (l.122-127).  Dilated
  (atrous) convs run as implicit GEMMs with dilated taps, transposed convs as strided
  data-gradient phases, the residual adds ride in the conv epilogues.
* MSResAttnRefine: the x / forward / backward streams share the encoder weights; the
  local-window attention (corrmap l.253-287 and the two neighbour weightings l.289-323)
  runs on the dvie_attn kernels (L2 normalisation, 5x9 correlation volume over both
  target maps, one softmax over the 90 entries, optional 3x5 average pooling
  (stage3_prop), per-map normalised low-resolution weighting, the weighted gather), all
  with their backward in the same plan.  Concats are channel slices of one buffer.
"""
import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import FlatParams, PlanFunction, PlanPool, precision_of
from .conv import Conv2d

WH, WW = 5, 9  # attention window (refine_nets.py:250-251)
NATT = E.rup(2 * WH * WW, 4)  # 90 window weights (+2 pad) per pixel


class ResnetBlock(nn.Module):
    """conv-LReLU-conv + input (refine_nets.py:14-24)."""

    def __init__(self, in_dim, out_dim, ks):
        super().__init__()
        self.conv = nn.Sequential(Conv2d(in_dim, out_dim, ks, stride=1, padding=ks // 2),
                                  nn.LeakyReLU(0.2, inplace=True),
                                  Conv2d(out_dim, out_dim, ks, stride=1, padding=ks // 2))


def _lrelu():
    return nn.LeakyReLU(0.2, inplace=True)


def _seq_conv_act(*convs):
    """nn.Sequential(conv, LReLU, conv, LReLU, ...) of the given convs."""
    layers = []
    for c in convs:
        layers += [c, _lrelu()]
    return nn.Sequential(*layers)


class _Lower:
    """Small helpers over an engine Graph (buffers named by a running counter)."""

    def __init__(self, g, trainable, tag):
        self.g, self.tr, self.tag, self.k = g, trainable, tag, 0

    def buf(self, H, W, C, name=""):
        self.k += 1
        return self.g.buffer(f"{self.tag}{self.k}.{name}", H, W, C)

    def conv(self, x, m, act=True, res=None, out=None, cmap=None, name=""):
        s, p, d, k = m.stride[0], m.padding[0], m.dilation[0], m.kernel_size[0]
        H = (x.H + 2 * p - d * (k - 1) - 1) // s + 1
        W = (x.W + 2 * p - d * (k - 1) - 1) // s + 1
        if out is None:
            out = E.R(self.buf(H, W, E.rup(m.out_channels, 8), name))
        self.g.conv(x, m, out, act=L.ACT_LRELU if act else L.ACT_NONE, res=res, cmap=cmap, trainable=self.tr,
                    name=name)
        return out

    def convT(self, x, m, name=""):
        out = E.R(self.buf(x.H * 2, x.W * 2, E.rup(m.out_channels, 8), name))
        self.g.convT(x, m, out, act=L.ACT_LRELU, trainable=self.tr, name=name)
        return out

    def res(self, x, blk, name=""):
        t = self.conv(x, blk.conv[0], name=name + ".conv.0")
        return self.conv(t, blk.conv[2], act=False, res=x, name=name + ".conv.2")

    def add(self, a, b, name=""):
        out = E.R(self.buf(a.H, a.W, a.c, name))
        self.g.fuse([a, b], out)
        return out

    def resize(self, x, H, W, detach=False, out=None, name=""):
        if out is None:
            out = E.R(self.buf(H, W, x.c, name))
        self.g.fuse([x], out, align=True, detach=detach)
        return out

    def copy(self, x, out):
        self.g.fuse([x], out)
        return out


class SRNRefine(FlatParams, nn.Module):
    """forward(input_rgb, input_seg, encoded_feat) -> [prediction per scale], coarsest first.
    input_rgb (B, 3, H, W), input_seg (B, 20, H, W), encoded_feat (B, 14, H, W); H and W
    multiples of 4 * 2^(n_scales - 1)."""

    def __init__(self, args):
        super().__init__()
        self.n_scales = getattr(args, "n_scales", 1)
        self.args = args
        self.input_layer = nn.Sequential(
            Conv2d(3 + 3 + 20 + 14, 32, 3, stride=1, padding=1), _lrelu(),
            Conv2d(32, 32, 3, stride=1, padding=1), _lrelu(),
            Conv2d(32, 64, 3, stride=1, padding=1), _lrelu(),
            ResnetBlock(64, 64, 3), ResnetBlock(64, 64, 3), ResnetBlock(64, 64, 3))
        self.encoder_1 = nn.Sequential(Conv2d(64, 128, 3, stride=2, padding=1), _lrelu(),
                                       ResnetBlock(128, 128, 3), ResnetBlock(128, 128, 3), ResnetBlock(128, 128, 3))
        self.encoder_2 = nn.Sequential(Conv2d(128, 256, 3, stride=2, padding=1), _lrelu(),
                                       ResnetBlock(256, 256, 3), ResnetBlock(256, 256, 3), ResnetBlock(256, 256, 3))
        self.bottle_dilated = _seq_conv_act(*[Conv2d(256, 256, 3, 1, d, d) for d in (1, 2, 4, 8)])
        self.hidden_comb = _seq_conv_act(Conv2d(512, 256, 3, 1, 1), Conv2d(256, 256, 3, 1, 1))
        self.decoder_2 = nn.Sequential(ResnetBlock(256, 256, 3), ResnetBlock(256, 256, 3), ResnetBlock(256, 256, 3),
                                       nn.ConvTranspose2d(256, 128, 4, stride=2, padding=1), _lrelu())
        self.decoder_1 = nn.Sequential(ResnetBlock(128, 128, 3), ResnetBlock(128, 128, 3), ResnetBlock(128, 128, 3),
                                       nn.ConvTranspose2d(128, 64, 4, stride=2, padding=1), _lrelu())
        self.output_layer = nn.Sequential(ResnetBlock(64, 64, 3), ResnetBlock(64, 64, 3), ResnetBlock(64, 64, 3),
                                          Conv2d(64, 32, 3, 1, padding=1), _lrelu(),
                                          Conv2d(32, 3, 3, 1, padding=1))
        self.dtype = precision_of(args)
        self._pool = PlanPool(self._build_plan)
        self._flatten()

    # input buffer: [pred 3 (+5) | rgb 3 (+5) | seg 20 (+4) | enc 14 (+2)] = 56 channels
    _CMAP = ([3, 4, 5] + [-1] * 5 + [0, 1, 2] + [-1] * 5 + list(range(6, 26)) + [-1] * 4 + list(range(26, 40))
             + [-1] * 2)

    def _lower(self, g, H, W, trainable):
        lw = _Lower(g, trainable, "srn")
        X = g.buffer("in_full", H, W, 56)
        g.input_nchw(E.R(X, 0, 8), "rgb", ext_c=3)   # the coarsest scale's "previous prediction" is rgb
        g.input_nchw(E.R(X, 8, 8), "rgb", ext_c=3)
        g.input_nchw(E.R(X, 16, 24), "seg", ext_c=20)
        g.input_nchw(E.R(X, 40, 16), "enc", ext_c=14)
        ns = self.n_scales
        pred = hidden = None
        for si in range(ns - 1, -1, -1):
            h, w = H >> si, W >> si
            coarsest = si == ns - 1
            if si == 0:
                Xs = E.R(X)
            else:
                Xs = lw.resize(E.R(X), h, w, name=f"in_s{si}")
            if not coarsest:  # previous prediction, 2x up and detached (refine_nets.py:111)
                lw.resize(pred, h, w, detach=True, out=E.R(Xs.buf, 0, 8))
            il = lw.conv(Xs, self.input_layer[0], cmap=self._CMAP, name="input_layer.0")
            il = lw.conv(il, self.input_layer[2], name="input_layer.2")
            il = lw.conv(il, self.input_layer[4], name="input_layer.4")
            for i in (6, 7, 8):
                il = lw.res(il, self.input_layer[i], f"input_layer.{i}")
            e1 = lw.conv(il, self.encoder_1[0], name="encoder_1.0")
            for i in (2, 3, 4):
                e1 = lw.res(e1, self.encoder_1[i], f"encoder_1.{i}")
            e2 = lw.conv(e1, self.encoder_2[0], name="encoder_2.0")
            for i in (2, 3, 4):
                e2 = lw.res(e2, self.encoder_2[i], f"encoder_2.{i}")
            bo = e2
            for i in range(4):
                bo = lw.conv(bo, self.bottle_dilated[2 * i], name=f"bottle_dilated.{2 * i}")
            HC = lw.buf(bo.H, bo.W, 512, "hidden_in")  # cat([bottle_out, last_hidden])
            lw.copy(bo, E.R(HC, 0, 256))
            if coarsest:
                lw.copy(bo, E.R(HC, 256, 256))
            else:
                lw.resize(hidden, bo.H, bo.W, out=E.R(HC, 256, 256))
            hc = lw.conv(E.R(HC), self.hidden_comb[0], name="hidden_comb.0")
            hidden = lw.conv(hc, self.hidden_comb[2], name="hidden_comb.2")
            d2 = lw.add(hidden, e2, "dec2_in")
            for i in (0, 1, 2):
                d2 = lw.res(d2, self.decoder_2[i], f"decoder_2.{i}")
            d2 = lw.convT(d2, self.decoder_2[3], "decoder_2.3")
            d1 = lw.add(d2, e1, "dec1_in")
            for i in (0, 1, 2):
                d1 = lw.res(d1, self.decoder_1[i], f"decoder_1.{i}")
            d1 = lw.convT(d1, self.decoder_1[3], "decoder_1.3")
            o = lw.add(d1, il, "out_in")
            for i in (0, 1, 2):
                o = lw.res(o, self.output_layer[i], f"output_layer.{i}")
            o = lw.conv(o, self.output_layer[3], name="output_layer.3")
            pred = lw.conv(o, self.output_layer[5], act=False, name="output_layer.5")
            g.output_nchw(f"pred{ns - 1 - si}", pred, 3)
        return g

    def _build_plan(self, key):
        n, H, W, dtype, trainable, dev = key
        g = E.Graph(dtype)
        self._lower(g, H, W, trainable)
        return g.compile(n, dev, backward=trainable)

    def _on_moved(self):
        self._pool.clear()

    def run_forward(self, inputs, train):
        rgb, seg, enc = inputs
        L.require_gpu(rgb)
        n, _, H, W = rgb.shape
        m = 4 << (self.n_scales - 1)
        if H % m or W % m:
            raise ValueError(f"SRNRefine: H and W must be multiples of {m} (n_scales={self.n_scales})")
        trainable = bool(train) and any(p.requires_grad for p in self.parameters())
        plan = self._pool.acquire((n, H, W, self.dtype, trainable, rgb.device))
        plan.set_input("rgb", rgb)
        plan.set_input("seg", seg)
        plan.set_input("enc", enc)
        outs = []
        for i in range(self.n_scales):
            s = self.n_scales - 1 - i
            t = torch.empty((n, 3, H >> s, W >> s), dtype=torch.float32, device=rgb.device)
            plan.set_output_nchw(f"pred{i}", t)
            outs.append(t)
        plan.run_forward()
        self.last_plan = plan
        return plan, tuple(outs)

    def run_backward(self, plan, inputs, grads, needs):
        plan.set_param_grads(self.grad_views())
        for i, gr in enumerate(grads):
            s = self.n_scales - 1 - i
            n, _, H, W = inputs[0].shape
            if gr is None:
                gr = torch.zeros((n, 3, H >> s, W >> s), dtype=torch.float32, device=inputs[0].device)
            plan.set_output_grad(f"pred{i}", gr.float())
        plan.run_backward()
        return [None, None, None]

    def forward(self, input_rgb, input_seg=None, encoded_feat=None):
        outs = PlanFunction.apply(self, 3, input_rgb.float().detach(), input_seg.float().detach(),
                                  encoded_feat.float().detach(), *self._flat_params)
        return list(outs) if isinstance(outs, tuple) else [outs]


class MSResAttnRefine(FlatParams, nn.Module):
    """forward(coarse_img, coarse_seg, neighbors_img, neighbors_seg) -> (outputs per scale,
    flow maps per scale), coarsest first; flow maps (B, 2, 2, h, w) float on the CPU as the
    reference returns them.  H, W multiples of 4 * 2^(n_scales - 1)."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.n_scales = getattr(args, "n_scales", 1)
        self.input_layer = _seq_conv_act(Conv2d(3 + 20, 32, 3, 1, 1), Conv2d(32, 64, 3, 1, 1))
        self.attn_input_layer = _seq_conv_act(Conv2d(64, 64, 3, 1, 1), Conv2d(64, 64, 3, 1, 1))
        self.attn_encoder_1 = _seq_conv_act(Conv2d(64, 64, 3, 2, 1), Conv2d(64, 64, 3, 1, 1))
        self.attn_encoder_2 = _seq_conv_act(Conv2d(64, 128, 3, 2, 1), Conv2d(128, 128, 3, 1, 1))
        self.attn_fuse_layer = _seq_conv_act(Conv2d(128, 128, 3, 1, 1), Conv2d(128, 128, 3, 1, 1))
        self.attn_img_fuse_layer = _seq_conv_act(Conv2d(256, 128, 3, 1, 1), Conv2d(128, 128, 3, 1, 1))
        self.img_input_layer = _seq_conv_act(Conv2d(64 * 3, 64, 3, 1, 1), Conv2d(64, 64, 3, 1, 1))
        self.img_encoder_1 = _seq_conv_act(Conv2d(64, 64, 3, 2, 1), Conv2d(64, 64, 3, 1, 1))
        self.img_encoder_2 = _seq_conv_act(Conv2d(64, 128, 3, 2, 1), Conv2d(128, 128, 3, 1, 1))
        self.img_atrous_layer = _seq_conv_act(*[Conv2d(128, 128, 3, 1, d, d) for d in (1, 2, 4, 8)])
        self.img_fuse_layer = _seq_conv_act(Conv2d(256, 128, 3, 1, 1), Conv2d(128, 128, 3, 1, 1))
        self.decoder_2 = nn.Sequential(nn.ConvTranspose2d(128, 64, 4, 2, 1), _lrelu(), ResnetBlock(64, 64, 3))
        self.decoder_1 = nn.Sequential(nn.ConvTranspose2d(64, 64, 4, 2, 1), _lrelu(), ResnetBlock(64, 64, 3))
        self.output_layer = nn.Sequential(Conv2d(64, 64, 3, 1, 1), _lrelu(), Conv2d(64, 32, 3, 1, 1), _lrelu(),
                                          Conv2d(32, 3, 3, 1, 1))
        self.w = WW
        self.h = WH
        self.dtype = precision_of(args)
        self._pool = PlanPool(self._build_plan)
        self._flatten()

    # stream input [img 3 (+1) | seg 20] -> conv input order [img 3, seg 20]
    _CMAP = [0, 1, 2, -1] + list(range(3, 23))

    def _two(self, lw, x, seq, base):
        x = lw.conv(x, seq[0], name=f"{base}.0")
        return lw.conv(x, seq[2], name=f"{base}.2")

    def _lower(self, g, H, W, trainable, prop):
        lw = _Lower(g, trainable, "att")
        full = {}
        for s_, key, sk, c0 in (("x", "img", "seg", 0), ("f", "nimg", "nseg", 0), ("b", "nimg", "nseg", 1)):
            X = g.buffer(f"in_{s_}", H, W, 24)
            g.input_nchw(E.R(X, 0, 4), key, ext_c0=3 * c0, ext_c=3)
            g.input_nchw(E.R(X, 4, 20), sk, ext_c0=20 * c0, ext_c=20)
            full[s_] = E.R(X)
        ns = self.n_scales
        probs, self_sims = [], []
        for si in range(ns - 1, -1, -1):
            h, w = H >> si, W >> si
            il, a2 = {}, {}
            for s_ in ("x", "f", "b"):
                x = full[s_] if si == 0 else lw.resize(full[s_], h, w, name=f"in_{s_}{si}")
                t = lw.conv(x, self.input_layer[0], cmap=self._CMAP, name="input_layer.0")
                il[s_] = lw.conv(t, self.input_layer[2], name="input_layer.2")
                t = self._two(lw, il[s_], self.attn_input_layer, "attn_input_layer")
                t = self._two(lw, t, self.attn_encoder_1, "attn_encoder_1")
                a2[s_] = self._two(lw, t, self.attn_encoder_2, "attn_encoder_2")
            ah, aw = a2["x"].H, a2["x"].W
            fw, bw = a2["f"], a2["b"]
            if si != ns - 1:  # low-resolution prob maps weight the targets (l.365-372)
                for pk in probs:
                    up = lw.resize(pk, ah, aw, name="low_prob")
                    wn = E.R(lw.buf(ah, aw, NATT, "low_wnorm"))
                    g.wnorm(up, wn, 2, WH, WW)
                    nf = E.R(lw.buf(ah, aw, 128, "low_fw"))
                    g.gather(wn, [fw], nf, 0, 2, WH, WW)
                    nb = E.R(lw.buf(ah, aw, 128, "low_bw"))
                    g.gather(wn, [bw], nb, 1, 2, WH, WW)
                    fw, bw = nf, nb
                fw = self._two(lw, fw, self.attn_fuse_layer, "attn_fuse_layer")
                bw = self._two(lw, bw, self.attn_fuse_layer, "attn_fuse_layer")
            # corrmap (l.253-287)
            xn, fn, bn = (E.R(lw.buf(ah, aw, 128, n)) for n in ("xn", "fn", "bn"))
            g.l2norm(a2["x"], xn)
            g.l2norm(fw, fn)
            g.l2norm(bw, bn)
            sim = E.R(lw.buf(ah, aw, NATT, "sim"))
            g.corr(xn, [fn, bn], sim, WH, WW)
            self_sims.append(sim)
            prob = E.R(lw.buf(ah, aw, NATT, "prob"))
            g.softmax(sim, prob, 2, WH, WW)
            if prop:
                pp = E.R(lw.buf(ah, aw, NATT, "prob_prop"))
                g.apool(prob, pp, 3, 5)
                prob = pp
            probs.append(prob)
            # attention-weighted neighbour features + attention image fuse (l.379-381)
            AF = lw.buf(ah, aw, 256, "attn_fuse_in")
            lw.copy(a2["x"], E.R(AF, 0, 128))
            g.gather(prob, [a2["f"], a2["b"]], E.R(AF, 128, 128), 0, 2, WH, WW)
            af = self._two(lw, E.R(AF), self.attn_img_fuse_layer, "attn_img_fuse_layer")
            # image module (l.384-389)
            II = lw.buf(h, w, 192, "img_in")
            for k, s_ in enumerate(("x", "f", "b")):
                lw.copy(il[s_], E.R(II, 64 * k, 64))
            ii = self._two(lw, E.R(II), self.img_input_layer, "img_input_layer")
            ie1 = self._two(lw, ii, self.img_encoder_1, "img_encoder_1")
            ie2 = self._two(lw, ie1, self.img_encoder_2, "img_encoder_2")
            FU = lw.buf(ah, aw, 256, "fuse_in")
            t = ie2
            for i in range(3):
                t = lw.conv(t, self.img_atrous_layer[2 * i], name=f"img_atrous_layer.{2 * i}")
            lw.conv(t, self.img_atrous_layer[6], out=E.R(FU, 0, 128), name="img_atrous_layer.6")
            lw.copy(af, E.R(FU, 128, 128))
            fu = self._two(lw, E.R(FU), self.img_fuse_layer, "img_fuse_layer")
            d2 = lw.convT(fu, self.decoder_2[0], "decoder_2.0")
            d2 = lw.res(d2, self.decoder_2[2], "decoder_2.2")
            d1 = lw.convT(lw.add(d2, ie1, "dec1_in"), self.decoder_1[0], "decoder_1.0")
            d1 = lw.res(d1, self.decoder_1[2], "decoder_1.2")
            o = lw.add(d1, ii, "out_in")
            o = lw.conv(o, self.output_layer[0], name="output_layer.0")
            o = lw.conv(o, self.output_layer[2], name="output_layer.2")
            o = lw.conv(o, self.output_layer[4], act=False, name="output_layer.4")
            g.output_nchw(f"out{ns - 1 - si}", o, 3)
        g.sims = self_sims
        return g

    def _build_plan(self, key):
        n, H, W, dtype, trainable, prop, dev = key
        g = E.Graph(dtype)
        self._lower(g, H, W, trainable, prop)
        plan = g.compile(n, dev, backward=trainable)
        plan.sims = g.sims
        return plan

    def _on_moved(self):
        self._pool.clear()

    def run_forward(self, inputs, train):
        img, seg, nimg, nseg = inputs
        L.require_gpu(img)
        n, _, H, W = img.shape
        m = 4 << (self.n_scales - 1)
        if H % m or W % m:
            raise ValueError(f"MSResAttnRefine: H and W must be multiples of {m} (n_scales={self.n_scales})")
        trainable = bool(train) and any(p.requires_grad for p in self.parameters())
        prop = bool(getattr(self.args, "stage3_prop", False))
        plan = self._pool.acquire((n, H, W, self.dtype, trainable, prop, img.device))
        for k, t in (("img", img), ("seg", seg), ("nimg", nimg), ("nseg", nseg)):
            plan.set_input(k, t)
        outs = []
        for i in range(self.n_scales):
            s = self.n_scales - 1 - i
            t = torch.empty((n, 3, H >> s, W >> s), dtype=torch.float32, device=img.device)
            plan.set_output_nchw(f"out{i}", t)
            outs.append(t)
        plan.run_forward()
        self.last_plan = plan
        return plan, tuple(outs)

    def run_backward(self, plan, inputs, grads, needs):
        plan.set_param_grads(self.grad_views())
        n, _, H, W = inputs[0].shape
        for i, gr in enumerate(grads):
            s = self.n_scales - 1 - i
            if gr is None:
                gr = torch.zeros((n, 3, H >> s, W >> s), dtype=torch.float32, device=inputs[0].device)
            plan.set_output_grad(f"out{i}", gr.float())
        plan.run_backward()
        return [None, None, None, None]

    @staticmethod
    def flow_maps(plan):
        """corrmap's flow maps (refine_nets.py:273-279) from the similarity buffers of the
        last forward: per map, window argmax k -> (k // h, k % h) - (w//2, h//2), the
        reference's own index decomposition; float (B, 2, 2, h, w).  They stay on the
        device (the reference moves them to the CPU; a device-to-host copy inside a step
        would break its hipGraph capture): callers that visualise them call .cpu()."""
        flows = []
        for sim in plan.sims:
            t = sim.buf.t[..., :2 * WH * WW]
            n, h, w = t.shape[:3]
            idx = t.reshape(n, h, w, 2, WH * WW).argmax(-1).permute(0, 3, 1, 2)  # (B, 2, h, w)
            flows.append(torch.stack([idx // WH - WW // 2, idx % WH - WH // 2], 2).float())
        return flows

    def forward(self, coarse_img, coarse_seg, neighbors_img, neighbors_seg):
        outs = PlanFunction.apply(self, 4, coarse_img.float().detach(), coarse_seg.float().detach(),
                                  neighbors_img.float().detach(), neighbors_seg.float().detach(), *self._flat_params)
        outs = list(outs) if isinstance(outs, tuple) else [outs]
        return outs, self.flow_maps(self.last_plan)
