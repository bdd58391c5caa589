"""Oracle: HRNet coarse generator (reference nets/HRNet.py:339-601), functional CPU fp32.

`conv_specs` lists the convolutions in the order the reference constructs them
(nn.Conv2d default init consumes the global RNG in that order, so building them in this
order under torch.manual_seed(s) reproduces the reference's initial weights);
`init_params` builds the state dict; `forward` restates HRNet.forward (l.524-601) with
F.conv2d / F.leaky_relu / F.elu / F.interpolate.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

STAGES = {False: [[64, 128], [64, 128, 256]], True: [[64, 128], [64, 128, 256], [64, 128, 256, 512]]}


def conv_specs(n_frames=2, rgb_out=3, seg_out=20, large=False, extra_in=0):
    """[(name, cin, cout, k, stride, pad, bias)] in reference construction order
    (extra_in: VAEHRNet's decoded feature channels in the stem concat, HRNet.py:718-720)."""
    S = []

    def add(name, cin, cout, k, s=1, p=None, bias=False):
        S.append((name, cin, cout, k, s, (k // 2) if p is None else p, bias))

    # seg_encoder (l.358-364)
    add("seg_encoder.0", 20, 32, 3, bias=True)
    add("seg_encoder.2", 32, 32, 3, bias=True)
    add("seg_encoder.4", 32, 4, 3, bias=True)
    # stem (l.367-371)
    add("conv1", 7 * n_frames + extra_in, 64, 3, bias=True)
    add("conv2", 64, 64, 3, bias=True)
    # layer1: _make_layer builds the downsample before the first Bottleneck (l.479-495)
    add("layer1.0.downsample.0", 64, 256, 1)
    for b in range(4):
        add(f"layer1.{b}.conv1", 64 if b == 0 else 256, 64, 1)
        add(f"layer1.{b}.conv2", 64, 64, 3)
        add(f"layer1.{b}.conv3", 64, 256, 1)
    pre = [256]
    for si, chans in enumerate(STAGES[large]):
        t = f"transition{si + 1}"
        for i, c in enumerate(chans):  # _make_transition_layer (l.444-477)
            if i < len(pre):
                if c != pre[i]:
                    add(f"{t}.{i}.0", pre[i], c, 3)
            else:
                for j in range(i + 1 - len(pre)):
                    add(f"{t}.{i}.{j}.0", pre[-1], c if j == i - len(pre) else pre[-1], 3, 2)
        st = f"stage{si + 2}.0"
        nb = len(chans)
        for i in range(nb):  # _make_branches (l.126-152)
            for b in range(4):
                add(f"{st}.branches.{i}.{b}.conv1", chans[i], chans[i], 3)
                add(f"{st}.branches.{i}.{b}.conv2", chans[i], chans[i], 3)
        for i in range(nb):  # _make_fuse_layers (l.154-198)
            for j in range(nb):
                if j > i:
                    add(f"{st}.fuse_layers.{i}.{j}.0", chans[j], chans[i], 1)
                elif j < i:
                    for k in range(i - j):
                        last = k == i - j - 1
                        add(f"{st}.fuse_layers.{i}.{j}.{k}.0", chans[j], chans[i] if last else chans[j], 3, 2)
        pre = chans
    last = sum(pre)
    add("rgb_layer.0", last, last, 1, bias=True)
    add("rgb_layer.2", last, rgb_out, 3, bias=True)
    add("seg_layer.0", last, last, 1, bias=True)
    add("seg_layer.2", last, seg_out, 3, bias=True)
    return S


def init_params(seed=1024, sd=None, **kw):
    """State dict with the reference's seeded nn.Conv2d initialisation (seed None: continue
    the current RNG stream, adding to `sd`)."""
    if seed is not None:
        torch.manual_seed(seed)
    sd = {} if sd is None else sd
    for name, cin, cout, k, s, p, bias in conv_specs(**kw):
        m = nn.Conv2d(cin, cout, k, s, p, bias=bias)
        sd[name + ".weight"] = m.weight.detach().clone()
        if bias:
            sd[name + ".bias"] = m.bias.detach().clone()
    return sd


def _conv(P, name, x, s=1, p=None):
    w = P[name + ".weight"]
    k = w.shape[-1]
    return F.conv2d(x, w, P.get(name + ".bias"), stride=s, padding=k // 2 if p is None else p)


def _lrelu(x, masks=None, name=None):
    """LeakyReLU(0.2); with `masks` (plan activation-buffer name -> bool NCHW tensor of the
    branch the implementation under test took, Plan.activation_signs) the branch decisions
    are imposed, so that an fp64 oracle can check an fp32 implementation's gradients without
    LeakyReLU kink flips (an activation within rounding of zero taking the other branch)
    dominating the comparison.  `name` may carry a channel slice: (buffer, c0, c)."""
    if masks is None or name is None:
        return F.leaky_relu(x, 0.2)
    key, c0, c = name if isinstance(name, tuple) else (name, 0, None)
    if key not in masks:
        return F.leaky_relu(x, 0.2)
    m = masks[key]
    m = m[:, c0:c0 + (x.shape[1] if c is None else c)].to(x.device)
    return torch.where(m, x, 0.2 * x)


def forward(P, inp, n_frames=2, large=False, taps=None, pre=None, masks=None):
    """HRNet.forward (nets/HRNet.py:524-601) for syn_type 'inter' (and 'extra' without
    inpainting).  inp: (B, 3F + 20F, H, W).  Returns (rgb, seg_logits).  pre: VAEHRNet's
    decoded feature, leading the stem concat (HRNet.py:997).  masks: imposed LeakyReLU
    branches (see _lrelu), keyed by the HRNet plan's activation buffer names."""
    M = masks
    F_ = n_frames
    segs = [inp[:, 3 * F_ + 20 * k: 3 * F_ + 20 * (k + 1)] for k in range(F_)]
    enc = []
    for s in segs:  # seg_encoder: conv-ELU-conv-ELU-conv
        h = F.elu(_conv(P, "seg_encoder.0", s))
        h = F.elu(_conv(P, "seg_encoder.2", h))
        enc.append(_conv(P, "seg_encoder.4", h))
    x = torch.cat(([pre] if pre is not None else []) + [inp[:, :3 * F_]] + enc, 1)
    x = _lrelu(_conv(P, "conv1", x), M, "stem1")
    x = _lrelu(_conv(P, "conv2", x), M, "stem2")
    for b in range(4):  # Bottleneck (l.66-85)
        r = _conv(P, "layer1.0.downsample.0", x) if b == 0 else x
        o = _lrelu(_conv(P, f"layer1.{b}.conv1", x), M, f"layer1.{b}.a")
        o = _lrelu(_conv(P, f"layer1.{b}.conv2", o), M, f"layer1.{b}.b")
        o = _conv(P, f"layer1.{b}.conv3", o)
        x = _lrelu(o + r, M, f"layer1.{b}.out")
    y_list = [x]
    pre = [256]
    for si, chans in enumerate(STAGES[large]):
        t = f"transition{si + 1}"
        x_list = []
        for i, c in enumerate(chans):
            src = x if si == 0 else y_list[-1]
            if i < len(pre):
                if c != pre[i]:
                    x_list.append(_lrelu(_conv(P, f"{t}.{i}.0", src), M, f"trans{si}.{i}.0"))
                else:
                    x_list.append(y_list[i])
            else:
                h = src
                for j in range(i + 1 - len(pre)):
                    h = _lrelu(_conv(P, f"{t}.{i}.{j}.0", h, s=2), M, f"trans{si}.{i}.{j}")
                x_list.append(h)
        st = f"stage{si + 2}.0"
        nb = len(chans)
        xs = []
        for i in range(nb):  # BasicBlock (l.28-44)
            h = x_list[i]
            for b in range(4):
                o = _lrelu(_conv(P, f"{st}.branches.{i}.{b}.conv1", h), M, f"{st}.branches.{i}.{b}.h")
                if taps is not None:
                    taps[f"{st}.branches.{i}.{b}.h"] = o
                o = _conv(P, f"{st}.branches.{i}.{b}.conv2", o)
                h = _lrelu(o + h, M, f"{st}.branches.{i}.{b}.out")
                if taps is not None:
                    taps[f"{st}.branches.{i}.{b}.out"] = h
            xs.append(h)
        ys = []
        for i in range(nb):  # HighResolutionModule.forward fuse (l.211-225)
            if i == 0:
                y = xs[0]
            else:
                y = _fuse_down(P, st, i, 0, xs[0], M)
            for j in range(1, nb):
                if i == j:
                    y = y + xs[j]
                elif j > i:
                    y = y + F.interpolate(_conv(P, f"{st}.fuse_layers.{i}.{j}.0", xs[j]),
                                          size=[xs[i].shape[-2], xs[i].shape[-1]], mode="bilinear",
                                          align_corners=False)
                else:
                    y = y + _fuse_down(P, st, i, j, xs[j], M)
            final = si == len(STAGES[large]) - 1
            # the plan writes the final stage's first fuse output into the concat buffer
            ys.append(_lrelu(y, M, ("cat", 0, y.shape[1]) if final and i == 0 else f"{st}.y{i}"))
        y_list = ys
        pre = chans
    x = y_list
    h0, w0 = x[0].shape[-2:]
    ups = [F.interpolate(t, size=(h0, w0), mode="bilinear", align_corners=False) for t in x[1:]]
    x = torch.cat([x[0]] + ups, 1)
    last = x.shape[1]
    stacked = M is not None and "heads_hidden" in M  # the plan's stacked 448 -> 896 head conv
    rgb = _conv(P, "rgb_layer.2", _lrelu(_conv(P, "rgb_layer.0", x), M,
                                         ("heads_hidden", 0, last) if stacked else "rgb_hidden"))
    seg = _conv(P, "seg_layer.2", _lrelu(_conv(P, "seg_layer.0", x), M,
                                         ("heads_hidden", last, last) if stacked else "seg_hidden"))
    return rgb, seg


def _fuse_down(P, st, i, j, x, masks=None):
    for k in range(i - j):
        x = _conv(P, f"{st}.fuse_layers.{i}.{j}.{k}.0", x, s=2)
        if k != i - j - 1:
            x = _lrelu(x, masks, f"{st}.down.{i}.{j}.{k}")
    return x
