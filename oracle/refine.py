"""Oracle (test infrastructure only): the second-stage refinement nets, functional CPU.

  SRNRefine        reference nets/refine_nets.py:27-135
  MSResAttnRefine  reference nets/refine_nets.py:138-399 (corrmap l.253-287,
                   weight_neighbors_by_low_probmap l.289-311, weight_neighbors_by_probmap
                   l.313-323)
  InterRefineNet / InterStage3Net glue: reference nets/InterRefineNet.py:8-53

`srn_specs` / `attn_specs` list the layers in the order the reference constructs them
(nn.Conv2d / nn.ConvTranspose2d default init draws from the global RNG in that order), so
`init_params(None, ...)` right after the coarse HRNet's init reproduces the reference's
initial weights.  The forward passes restate the reference's math with F.conv2d,
F.conv_transpose2d and F.interpolate; the local-window ops are written out as explicit
shifted-window sums.  Pinned by tests/golden/refine.npz (G11/G12, make_golden.py).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import hrnet as H

WH, WW = 5, 9  # attention window rows / cols (refine_nets.py:250-251)


def _res_block(S, name, c):
    S.append((name + ".conv.0", "c", c, c, 3, 1, 1, 1))
    S.append((name + ".conv.2", "c", c, c, 3, 1, 1, 1))


def srn_specs():
    """[(name, kind c|t, cin, cout, k, stride, pad, dilation)] in construction order."""
    S = []
    c = lambda n, ci, co, k=3, s=1, p=1, d=1: S.append((n, "c", ci, co, k, s, p, d))  # noqa: E731
    c("input_layer.0", 3 + 3 + 20 + 14, 32)
    c("input_layer.2", 32, 32)
    c("input_layer.4", 32, 64)
    for i in (6, 7, 8):
        _res_block(S, f"input_layer.{i}", 64)
    c("encoder_1.0", 64, 128, s=2)
    for i in (2, 3, 4):
        _res_block(S, f"encoder_1.{i}", 128)
    c("encoder_2.0", 128, 256, s=2)
    for i in (2, 3, 4):
        _res_block(S, f"encoder_2.{i}", 256)
    for i, d in enumerate((1, 2, 4, 8)):
        c(f"bottle_dilated.{2 * i}", 256, 256, p=d, d=d)
    c("hidden_comb.0", 512, 256)
    c("hidden_comb.2", 256, 256)
    for i in (0, 1, 2):
        _res_block(S, f"decoder_2.{i}", 256)
    S.append(("decoder_2.3", "t", 256, 128, 4, 2, 1, 1))
    for i in (0, 1, 2):
        _res_block(S, f"decoder_1.{i}", 128)
    S.append(("decoder_1.3", "t", 128, 64, 4, 2, 1, 1))
    for i in (0, 1, 2):
        _res_block(S, f"output_layer.{i}", 64)
    c("output_layer.3", 64, 32)
    c("output_layer.5", 32, 3)
    return S


def attn_specs():
    S = []
    c = lambda n, ci, co, s=1, p=1, d=1: S.append((n, "c", ci, co, 3, s, p, d))  # noqa: E731
    c("input_layer.0", 23, 32)
    c("input_layer.2", 32, 64)
    c("attn_input_layer.0", 64, 64)
    c("attn_input_layer.2", 64, 64)
    c("attn_encoder_1.0", 64, 64, s=2)
    c("attn_encoder_1.2", 64, 64)
    c("attn_encoder_2.0", 64, 128, s=2)
    c("attn_encoder_2.2", 128, 128)
    c("attn_fuse_layer.0", 128, 128)
    c("attn_fuse_layer.2", 128, 128)
    c("attn_img_fuse_layer.0", 256, 128)
    c("attn_img_fuse_layer.2", 128, 128)
    c("img_input_layer.0", 192, 64)
    c("img_input_layer.2", 64, 64)
    c("img_encoder_1.0", 64, 64, s=2)
    c("img_encoder_1.2", 64, 64)
    c("img_encoder_2.0", 64, 128, s=2)
    c("img_encoder_2.2", 128, 128)
    for i, d in enumerate((1, 2, 4, 8)):
        c(f"img_atrous_layer.{2 * i}", 128, 128, p=d, d=d)
    c("img_fuse_layer.0", 256, 128)
    c("img_fuse_layer.2", 128, 128)
    S.append(("decoder_2.0", "t", 128, 64, 4, 2, 1, 1))
    _res_block(S, "decoder_2.2", 64)
    S.append(("decoder_1.0", "t", 64, 64, 4, 2, 1, 1))
    _res_block(S, "decoder_1.2", 64)
    c("output_layer.0", 64, 64)
    c("output_layer.2", 64, 32)
    c("output_layer.4", 32, 3)
    return S


def init_params(seed, specs, sd=None):
    """Seeded nn.Conv2d / nn.ConvTranspose2d init in construction order (seed None:
    continue the current RNG stream)."""
    if seed is not None:
        torch.manual_seed(seed)
    sd = {} if sd is None else sd
    for name, kind, ci, co, k, s, p, d in specs:
        m = nn.Conv2d(ci, co, k, s, p, d) if kind == "c" else nn.ConvTranspose2d(ci, co, k, s, p)
        sd[name + ".weight"] = m.weight.detach().clone()
        sd[name + ".bias"] = m.bias.detach().clone()
    return sd


def _geo(specs):
    return {name: (kind, s, p, d) for name, kind, ci, co, k, s, p, d in specs}


def _lrelu(x):
    return F.leaky_relu(x, 0.2)


def _up(x, size=None, scale=None):
    return F.interpolate(x, size=size, scale_factor=scale, mode="bilinear", align_corners=True)


class _Net:
    """masks: the implementation's LeakyReLU branches, one bool NCHW tensor per activation in
    the order this restatement applies them (Plan.activation_list), imposed on the oracle so
    an fp64 evaluation follows the same branches (see hrnet._lrelu)."""

    def __init__(self, P, specs, masks=None):
        self.P, self.g = P, _geo(specs)
        self.masks = None if masks is None else iter(masks)

    def act(self, x):
        if self.masks is None:
            return _lrelu(x)
        m = next(self.masks)[:, :x.shape[1]].to(x.device)
        assert m.shape == x.shape, (m.shape, x.shape)
        return torch.where(m, x, 0.2 * x)

    def done(self):
        assert self.masks is None or next(self.masks, None) is None, "unused activation masks"

    def conv(self, name, x):
        kind, s, p, d = self.g[name]
        w, b = self.P[name + ".weight"], self.P[name + ".bias"]
        if kind == "t":
            return F.conv_transpose2d(x, w, b, stride=s, padding=p)
        return F.conv2d(x, w, b, stride=s, padding=p, dilation=d)

    def res(self, name, x):  # ResnetBlock: conv-LReLU-conv + input (refine_nets.py:14-24)
        return self.conv(name + ".conv.2", self.act(self.conv(name + ".conv.0", x))) + x

    def seq(self, names_acts, x):
        for n, act in names_acts:
            x = self.conv(n, x) if not n.endswith("!res") else self.res(n[:-4], x)
            if act:
                x = self.act(x)
        return x


def srn_forward(P, input_rgb, input_seg, encoded_feat, n_scales, masks=None):
    """SRNRefine.forward: per scale (coarsest first) input [rgb, previous prediction
    (2x up, detached), seg + encoded features] at that scale -> prediction; the hidden
    bottleneck state is carried (2x up, not detached) to the next scale."""
    N = _Net(P, srn_specs(), masks)
    others = torch.cat([input_seg, encoded_feat], 1)
    preds, hidden = [], []
    for si in range(n_scales - 1, -1, -1):
        scale = 1 / (2 ** si)
        ori = _up(input_rgb, scale=scale)
        coarsest = si == n_scales - 1
        pred_in = ori if coarsest else _up(preds[-1].detach(), scale=2)
        x = torch.cat([ori, pred_in, _up(others, scale=scale)], 1)
        il = N.seq([("input_layer.0", 1), ("input_layer.2", 1), ("input_layer.4", 1), ("input_layer.6!res", 0),
                    ("input_layer.7!res", 0), ("input_layer.8!res", 0)], x)
        e1 = N.seq([("encoder_1.0", 1)] + [(f"encoder_1.{i}!res", 0) for i in (2, 3, 4)], il)
        e2 = N.seq([("encoder_2.0", 1)] + [(f"encoder_2.{i}!res", 0) for i in (2, 3, 4)], e1)
        bo = N.seq([(f"bottle_dilated.{2 * i}", 1) for i in range(4)], e2)
        last = bo if coarsest else _up(hidden[-1], scale=2)
        hc = N.seq([("hidden_comb.0", 1), ("hidden_comb.2", 1)], torch.cat([bo, last], 1))
        hidden.append(hc)
        d2 = N.seq([(f"decoder_2.{i}!res", 0) for i in (0, 1, 2)] + [("decoder_2.3", 1)], hc + e2)
        d1 = N.seq([(f"decoder_1.{i}!res", 0) for i in (0, 1, 2)] + [("decoder_1.3", 1)], d2 + e1)
        out = N.seq([(f"output_layer.{i}!res", 0) for i in (0, 1, 2)] + [("output_layer.3", 1), ("output_layer.5", 0)],
                    d1 + il)
        preds.append(out)
    N.done()
    return preds


# ---------------- local-window attention (MSResAttnRefine) ----------------
def _neighbours(t, wh=WH, ww=WW):
    """(B, C, H, W) -> list over window entries k = i*ww + j of t shifted so that entry
    (y, x) holds t[y + i - wh//2, x + j - ww//2] (zero outside)."""
    B, C, Hh, Ww = t.shape
    tp = F.pad(t, (ww // 2, ww // 2, wh // 2, wh // 2))
    return [tp[:, :, i:i + Hh, j:j + Ww] for i in range(wh) for j in range(ww)]


def _unit(x):
    return x / x.norm(dim=1, keepdim=True)


def corrmap(x, t1, t2, prop):
    """-> prob (B, H, W, 2K) and flow (B, 2, 2, H, W) as corrmap (refine_nets.py:253-287):
    cosine similarity of x with the two target maps over the window, argmax per map
    (index // h, index % h, minus (w//2, h//2): the reference's own decomposition), one
    softmax over both maps' entries, optionally 3x5 average-pooled (stage3_prop)."""
    xn = _unit(x)
    sims = []
    for t in (t1, t2):
        nb = _neighbours(_unit(t))
        sims.append(torch.stack([(xn * n).sum(1) for n in nb], -1))  # (B, H, W, K)
    sim = torch.stack(sims, 1)  # (B, 2, H, W, K)
    idx = sim.argmax(-1)
    flow = torch.stack([idx // WH, idx % WH], 2).float()
    flow = flow - torch.tensor([WW // 2, WH // 2], dtype=flow.dtype).view(1, 1, 2, 1, 1)
    prob = torch.softmax(torch.cat([sim[:, 0], sim[:, 1]], -1), -1)
    if prop:
        prob = F.avg_pool2d(prob.permute(0, 3, 1, 2), (3, 5), 1, (1, 2), count_include_pad=False).permute(0, 2, 3, 1)
    return prob, flow


def weighted_neighbours(f1, f2, prob):
    """sum over both maps' window entries of prob * neighbour feature (l.313-323)."""
    K = WH * WW
    out = 0
    for m, f in enumerate((f1, f2)):
        for k, n in enumerate(_neighbours(f)):
            out = out + n * prob[..., m * K + k].unsqueeze(1)
    return out


def weighted_neighbours_low(f1, f2, prob):
    """per map, the prob-weighted neighbour sum divided by that map's prob sum (l.289-311)."""
    K = WH * WW
    outs = []
    for m, f in enumerate((f1, f2)):
        pm = prob[..., m * K:(m + 1) * K]
        s = 0
        for k, n in enumerate(_neighbours(f)):
            s = s + n * pm[..., k].unsqueeze(1)
        outs.append(s / pm.sum(-1).unsqueeze(1))
    return outs


def attn_forward(P, coarse_img, coarse_seg, neighbors_img, neighbors_seg, n_scales, prop, masks=None):
    """MSResAttnRefine.forward (refine_nets.py:325-399) -> (outputs per scale, flow maps)."""
    N = _Net(P, attn_specs(), masks)
    x_comb = torch.cat([coarse_img, coarse_seg], 1)
    f_comb = torch.cat([neighbors_img[:, :3], neighbors_seg[:, :20]], 1)
    b_comb = torch.cat([neighbors_img[:, 3:6], neighbors_seg[:, 20:40]], 1)
    probs, flows, outs = [], [], []
    enc = [("input_layer.0", 1), ("input_layer.2", 1)]
    att = [("attn_input_layer.0", 1), ("attn_input_layer.2", 1)]
    e1 = [("attn_encoder_1.0", 1), ("attn_encoder_1.2", 1)]
    e2 = [("attn_encoder_2.0", 1), ("attn_encoder_2.2", 1)]
    for si in range(n_scales - 1, -1, -1):
        scale = 1 / (2 ** si)
        streams = []
        for comb in (x_comb, f_comb, b_comb):
            c = _up(comb, scale=scale) if scale != 1 else comb
            il = N.seq(enc, c)
            ai = N.seq(att, il)
            streams.append((il, N.seq(e2, N.seq(e1, ai))))
        (x_il, x_a2), (f_il, f_a2), (b_il, b_a2) = streams
        fw, bw = f_a2, b_a2
        if si != n_scales - 1:
            for k in range(len(probs)):
                low = _up(probs[k].permute(0, 3, 1, 2), scale=2 ** (len(probs) - k)).permute(0, 2, 3, 1)
                fw, bw = weighted_neighbours_low(fw, bw, low)
            fw = N.seq([("attn_fuse_layer.0", 1), ("attn_fuse_layer.2", 1)], fw)
            bw = N.seq([("attn_fuse_layer.0", 1), ("attn_fuse_layer.2", 1)], bw)
        prob, flow = corrmap(x_a2, fw, bw, prop)
        probs.append(prob)
        flows.append(flow)
        nbw = weighted_neighbours(f_a2, b_a2, prob)
        af = N.seq([("attn_img_fuse_layer.0", 1), ("attn_img_fuse_layer.2", 1)], torch.cat([x_a2, nbw], 1))
        ii = N.seq([("img_input_layer.0", 1), ("img_input_layer.2", 1)], torch.cat([x_il, f_il, b_il], 1))
        ie1 = N.seq([("img_encoder_1.0", 1), ("img_encoder_1.2", 1)], ii)
        ie2 = N.seq([("img_encoder_2.0", 1), ("img_encoder_2.2", 1)], ie1)
        atr = N.seq([(f"img_atrous_layer.{2 * i}", 1) for i in range(4)], ie2)
        fu = N.seq([("img_fuse_layer.0", 1), ("img_fuse_layer.2", 1)], torch.cat([atr, af], 1))
        d2 = N.seq([("decoder_2.0", 1), ("decoder_2.2!res", 0)], fu)
        d1 = N.seq([("decoder_1.0", 1), ("decoder_1.2!res", 0)], d2 + ie1)
        outs.append(N.seq([("output_layer.0", 1), ("output_layer.2", 1), ("output_layer.4", 0)], d1 + ii))
    N.done()
    return outs, flows


def inter_refine_forward(Pc, Pr, x, seg, n_scales, Ps=None, prop=False, masks=None, rmasks=None, smasks=None):
    """InterRefineNet (Ps None) / InterStage3Net forward (nets/InterRefineNet.py:15-53),
    train split: coarse HRNet, softmax of its seg logits (detached), the coarse seg
    encoder re-run on both input segs (detached), SRNRefine on the clamped detached coarse
    image; refine outputs clamped to [-10, 10] (InterRefineNet) or [-1, 1] (InterStage3Net,
    which then runs the stage-3 net on the last refine output, clamped to [-10, 10]).
    masks / rmasks / smasks: imposed activation branches of the coarse / refine / stage-3 nets."""
    rgb, seg_out = H.forward(Pc, torch.cat([x, seg], 1), masks=masks)
    soft = torch.softmax(seg_out, 1).detach()

    def segenc(s):
        h = F.elu(F.conv2d(s, Pc["seg_encoder.0.weight"], Pc["seg_encoder.0.bias"], padding=1))
        h = F.elu(F.conv2d(h, Pc["seg_encoder.2.weight"], Pc["seg_encoder.2.bias"], padding=1))
        return F.conv2d(h, Pc["seg_encoder.4.weight"], Pc["seg_encoder.4.bias"], padding=1)

    enc = torch.cat([x, segenc(seg[:, :20]).detach(), segenc(seg[:, 20:40]).detach()], 1)
    refine = srn_forward(Pr, rgb.detach().clamp(-1, 1), soft, enc, n_scales, masks=rmasks)
    if Ps is None:
        return rgb, seg_out, [r.clamp(-10, 10) for r in refine]
    refine = [r.clamp(-1, 1) for r in refine]
    outs, flows = attn_forward(Ps, refine[-1].detach(), soft, x, seg, n_scales, prop, masks=smasks)
    return rgb, seg_out, refine, [o.clamp(-10, 10) for o in outs], flows
