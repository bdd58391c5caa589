"""HRNet coarse generator (InterNet/ExtraNet backbone) on the MI355X plan engine.

Module tree, construction order (hence seeded initialisation) and parameter names are
those of the reference nets/HRNet.py:15-601 (BasicBlock l.15-44, Bottleneck l.47-85,
HighResolutionModule l.88-227, HRNet l.339-601), so reference checkpoints load with
`load_state_dict` unchanged.  The forward/backward do not run these submodules one by
one: `_build_graph` lowers the whole network to one engine plan (HIP implicit-GEMM
convolutions with fused bias / residual / LeakyReLU / ELU epilogues, fused multi-scale
upsample-sums, gradient epilogues fused as described in engine.py).

Layout: activations NHWC in the compute dtype (fp32 parity mode or bf16), channel counts
padded to multiples of 8; the 14-channel stem input is laid out as
[segA(4) 0000 segB(4) 0000 rgb(6) 00] and the stem weights are packed to match.
"""
import os

import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import FlatParams, PlanFunction, PlanPool, precision_of
from .conv import Conv2d

BN_MOMENTUM = 0.01


def conv3x3(in_planes, out_planes, stride=1):
    return Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.relu = nn.LeakyReLU(0.2, inplace=False)
        self.conv2 = conv3x3(planes, planes)
        self.downsample = downsample
        self.stride = stride


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.conv3 = Conv2d(planes, planes * self.expansion, kernel_size=1, bias=False)
        self.relu = nn.LeakyReLU(0.2, inplace=False)
        self.downsample = downsample
        self.stride = stride


blocks_dict = {"BASIC": BasicBlock, "BOTTLENECK": Bottleneck}


class HighResolutionModule(nn.Module):
    def __init__(self, num_branches, blocks, num_blocks, num_inchannels, num_channels, fuse_method,
                 multi_scale_output=True):
        super().__init__()
        if not (num_branches == len(num_blocks) == len(num_channels) == len(num_inchannels)):
            raise ValueError("NUM_BRANCHES mismatch")
        self.num_inchannels = num_inchannels
        self.fuse_method = fuse_method
        self.num_branches = num_branches
        self.multi_scale_output = multi_scale_output
        self.block = blocks
        self.branches = self._make_branches(num_branches, blocks, num_blocks, num_channels)
        self.fuse_layers = self._make_fuse_layers()
        self.relu = nn.LeakyReLU(0.2, inplace=False)

    def _make_one_branch(self, i, block, num_blocks, num_channels, stride=1):
        downsample = None
        if stride != 1 or self.num_inchannels[i] != num_channels[i] * block.expansion:
            downsample = nn.Sequential(Conv2d(self.num_inchannels[i], num_channels[i] * block.expansion,
                                              kernel_size=1, stride=stride, bias=False))
        layers = [block(self.num_inchannels[i], num_channels[i], stride, downsample)]
        self.num_inchannels[i] = num_channels[i] * block.expansion
        for _ in range(1, num_blocks[i]):
            layers.append(block(self.num_inchannels[i], num_channels[i]))
        return nn.Sequential(*layers)

    def _make_branches(self, num_branches, block, num_blocks, num_channels):
        return nn.ModuleList([self._make_one_branch(i, block, num_blocks, num_channels)
                              for i in range(num_branches)])

    def _make_fuse_layers(self):
        if self.num_branches == 1:
            return None
        nb, nin = self.num_branches, self.num_inchannels
        fuse_layers = []
        for i in range(nb if self.multi_scale_output else 1):
            fuse_layer = []
            for j in range(nb):
                if j > i:
                    fuse_layer.append(nn.Sequential(Conv2d(nin[j], nin[i], 1, 1, 0, bias=False)))
                elif j == i:
                    fuse_layer.append(None)
                else:
                    convs = []
                    for k in range(i - j):
                        if k == i - j - 1:
                            convs.append(nn.Sequential(Conv2d(nin[j], nin[i], 3, 2, 1, bias=False)))
                        else:
                            convs.append(nn.Sequential(Conv2d(nin[j], nin[j], 3, 2, 1, bias=False),
                                                       nn.LeakyReLU(0.2, inplace=False)))
                    fuse_layer.append(nn.Sequential(*convs))
            fuse_layers.append(nn.ModuleList(fuse_layer))
        return nn.ModuleList(fuse_layers)

    def get_num_inchannels(self):
        return self.num_inchannels


class _Cfg(dict):
    __getattr__ = dict.__getitem__


def _stage(blocks, chans):
    return _Cfg(NUM_MODULES=1, NUM_BRANCHES=len(blocks), NUM_BLOCKS=blocks, NUM_CHANNELS=chans, BLOCK="BASIC",
                FUSE_METHOD="SUM")


# nets/HRNet.py:238-335
HIGH_RESOLUTION_NET = _Cfg(STAGE2=_stage([4, 4], [64, 128]), STAGE3=_stage([4, 4, 4], [64, 128, 256]))
HIGH4_RESOLUTION_NET = _Cfg(STAGE2=_stage([4, 4], [64, 128]), STAGE3=_stage([4, 4, 4], [64, 128, 256]),
                            STAGE4=_stage([4, 4, 4, 4], [64, 128, 256, 512]))


def _out_hw(conv, H, W):
    k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1


def _arg(args, name, default):
    return getattr(args, name, default) if args is not None else default


class HRNet(FlatParams, nn.Module):
    """Reference: nets/HRNet.py:339-601.  forward(input) -> (rgb, seg_logits)."""

    _stem_extra = 0  # VAEHRNet: channels of the decoded VAE feature in the stem concat

    def __init__(self, args):
        super().__init__()
        self._setup(args)
        self._build_trunk()
        self._finish()

    def _setup(self, args):
        self.args = args
        self.highres_large = bool(_arg(args, "highres_large", False))
        self._extra = HIGH4_RESOLUTION_NET if self.highres_large else HIGH_RESOLUTION_NET
        self.syn_type = _arg(args, "syn_type", "inter")
        self.npo = _arg(args, "num_pred_once", 1) if self.syn_type == "extra" else 1
        self.inpaint_mask = bool(_arg(args, "inpaint_mask", False)) and self.syn_type == "extra"
        self.fix_init = bool(_arg(args, "fix_init_frames", False)) and self.syn_type == "extra"
        self.seg_encode_dim = 4
        self.n_classes = 20
        if self.syn_type == "extra":
            self.rgb_out_dim = 3 * self.npo if not self.inpaint_mask else 4 * self.npo
        else:
            self.rgb_out_dim = 3
        self.seg_out_dim = 20 * self.npo if self.syn_type == "extra" else 20
        self.n_frames = 3 if self.fix_init else 2
        self.in_channel = (3 + self.seg_encode_dim) * self.n_frames

    def _build_trunk(self):
        extra = self._extra
        self.in_channel += self._stem_extra
        self.seg_encoder = nn.Sequential(
            Conv2d(self.n_classes, 32, 3, 1, 1), nn.ELU(),
            Conv2d(32, 32, 3, 1, 1), nn.ELU(),
            Conv2d(32, self.seg_encode_dim, 3, 1, 1))
        self.conv1 = Conv2d(self.in_channel, 64, kernel_size=3, stride=1, padding=1, bias=True)
        self.conv2 = Conv2d(64, 64, kernel_size=3, stride=1, padding=1, bias=True)
        self.relu = nn.LeakyReLU(0.2, inplace=False)
        self.layer1 = self._make_layer(Bottleneck, 64, 64, 4)

        self.stage2_cfg = extra["STAGE2"]
        nc = [c * blocks_dict[self.stage2_cfg["BLOCK"]].expansion for c in self.stage2_cfg["NUM_CHANNELS"]]
        self.transition1 = self._make_transition_layer([256], nc)
        self.stage2, pre = self._make_stage(self.stage2_cfg, nc)

        self.stage3_cfg = extra["STAGE3"]
        nc = [c * blocks_dict[self.stage3_cfg["BLOCK"]].expansion for c in self.stage3_cfg["NUM_CHANNELS"]]
        self.transition2 = self._make_transition_layer(pre, nc)
        self.stage3, pre = self._make_stage(self.stage3_cfg, nc)

        if self.highres_large:
            self.stage4_cfg = extra["STAGE4"]
            nc = [c * blocks_dict[self.stage4_cfg["BLOCK"]].expansion for c in self.stage4_cfg["NUM_CHANNELS"]]
            self.transition3 = self._make_transition_layer(pre, nc)
            self.stage4, pre = self._make_stage(self.stage4_cfg, nc, multi_scale_output=True)

        last = int(sum(pre))
        self.last_inp_channels = last
        self.rgb_layer = nn.Sequential(Conv2d(last, last, 1, 1, 0), nn.LeakyReLU(0.2, inplace=False),
                                       Conv2d(last, self.rgb_out_dim, 3, 1, 1))
        self.seg_layer = nn.Sequential(Conv2d(last, last, 1, 1, 0), nn.LeakyReLU(0.2, inplace=False),
                                       Conv2d(last, self.seg_out_dim, 3, 1, 1))

    def _finish(self):
        self.dtype = precision_of(self.args)
        self._pool = PlanPool(self._build_plan)
        self._flatten(order=self._backward_order())

    # ---- reference constructors (same module creation order) ----
    def _make_transition_layer(self, pre, cur):
        layers = []
        for i in range(len(cur)):
            if i < len(pre):
                if cur[i] != pre[i]:
                    layers.append(nn.Sequential(Conv2d(pre[i], cur[i], 3, 1, 1, bias=False),
                                                nn.LeakyReLU(0.2, inplace=False)))
                else:
                    layers.append(None)
            else:
                convs = []
                for j in range(i + 1 - len(pre)):
                    inc = pre[-1]
                    outc = cur[i] if j == i - len(pre) else inc
                    convs.append(nn.Sequential(Conv2d(inc, outc, 3, 2, 1, bias=False),
                                               nn.LeakyReLU(0.2, inplace=False)))
                layers.append(nn.Sequential(*convs))
        return nn.ModuleList(layers)

    def _make_layer(self, block, inplanes, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or inplanes != planes * block.expansion:
            downsample = nn.Sequential(Conv2d(inplanes, planes * block.expansion, kernel_size=1, stride=stride,
                                              bias=False))
        layers = [block(inplanes, planes, stride, downsample)]
        inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(inplanes, planes))
        return nn.Sequential(*layers)

    def _make_stage(self, cfg, num_inchannels, multi_scale_output=True):
        modules = []
        for i in range(cfg["NUM_MODULES"]):
            reset = not (not multi_scale_output and i == cfg["NUM_MODULES"] - 1)
            modules.append(HighResolutionModule(cfg["NUM_BRANCHES"], blocks_dict[cfg["BLOCK"]], cfg["NUM_BLOCKS"],
                                                num_inchannels, cfg["NUM_CHANNELS"], cfg["FUSE_METHOD"], reset))
            num_inchannels = modules[-1].get_num_inchannels()
        return nn.Sequential(*modules), num_inchannels

    # ---- plan lowering ----
    def _backward_order(self):
        """Parameters in the order the backward pass completes them (heads first)."""
        g = self._lower(E.Graph(torch.float32), 16, 16, dry=True)
        order = []
        for lay in reversed(g.layers):
            if isinstance(lay.m, E.StackedConv):
                order += lay.m.params()
                continue
            order.append(lay.m.weight)
            if lay.m.bias is not None:
                order.append(lay.m.bias)
        return order

    def _stem_cmap(self):
        """packed stem position -> reference input channel ([rgb(3F), seg_enc(4 each)])."""
        F = self.n_frames
        e = self._stem_extra  # VAEHRNet: the VAE feature leads the reference concat (l.991-997)
        cm = []
        for k in range(F):
            cm += [e + 3 * F + 4 * k + i for i in range(4)] + [-1] * 4
        cm += [e + i for i in range(3 * F)] + [-1] * (E.rup(3 * F, 8) - 3 * F)
        cm += list(range(e))  # packed last: [segA 0000 segB 0000 rgb 00 | vae]
        return cm

    def _trunk_params(self):
        """parameters the HRNet plan writes gradients for"""
        return self._flat_params

    def _lower(self, g, H, W, dry=False, xgrad=False, vgrad=False):
        A = L
        g.dry = dry
        rup = E.rup
        F = self.n_frames
        segs = []
        stem_c = 8 * F + rup(3 * F, 8) + self._stem_extra
        feat = g.buffer("feat", H, W, stem_c)
        for k in range(F):
            s_in = g.buffer(f"seg{k}_in", H, W, 24)
            g.input_nchw(E.R(s_in), "seg", ext_c0=20 * k, ext_c=20)
            e1 = g.buffer(f"seg{k}_e1", H, W, 32)
            g.conv(E.R(s_in), self.seg_encoder[0], E.R(e1), act=A.ACT_ELU, name="seg_encoder.0")
            e2 = g.buffer(f"seg{k}_e2", H, W, 32)
            g.conv(E.R(e1), self.seg_encoder[2], E.R(e2), act=A.ACT_ELU, name="seg_encoder.2")
            g.conv(E.R(e2), self.seg_encoder[4], E.R(feat, 8 * k, 8), name="seg_encoder.4")
            g.segenc_chain(g.ops[-3:])  # one fused forward launch (engine Plan._segenc_fwd)
        # xgrad: the frames input needs a gradient (ExtraTrainer rollout feeds a prediction back)
        g.input_nchw(E.R(feat, 8 * F, rup(3 * F, 8)), "x", ext_c=3 * F, requires_grad=xgrad)
        if self._stem_extra:  # decoded VAE feature (its gradient feeds the decoder backward)
            g.input_nchw(E.R(feat, 8 * F + rup(3 * F, 8), self._stem_extra), "vae", ext_c=self._stem_extra,
                         requires_grad=vgrad)
        s1 = g.buffer("stem1", H, W, 64)
        g.conv(E.R(feat), self.conv1, E.R(s1), act=A.ACT_LRELU, cmap=self._stem_cmap(), name="conv1")
        if getattr(self, "_export_stem", False):
            # the stem concat [frames, seg_encoder(seg_k)...] as a detached NCHW side output
            # (InterRefineNet's encoded_feat, nets/InterRefineNet.py:21-25)
            g.export_nchw("stem_x", E.R(feat, 8 * F, rup(3 * F, 8)), 3 * F)
            for k in range(F):
                g.export_nchw(f"stem_seg{k}", E.R(feat, 8 * k, 4), 4)
        s2 = g.buffer("stem2", H, W, 64)
        g.conv(E.R(s1), self.conv2, E.R(s2), act=A.ACT_LRELU, name="conv2")
        x = E.R(s2)
        for bi, blk in enumerate(self.layer1):
            x = self._bottleneck(g, blk, x, f"layer1.{bi}")
        # stages
        xs = [x]
        y_list = [x]
        trans = [self.transition1, self.transition2] + ([self.transition3] if self.highres_large else [])
        stages = [self.stage2, self.stage3] + ([self.stage4] if self.highres_large else [])
        for si, (tr, st) in enumerate(zip(trans, stages)):
            x_list = []
            for i, t in enumerate(tr):
                if t is None:
                    x_list.append(y_list[i])
                    continue
                # reference: transition1[i](x) (nets/HRNet.py:548-553), later transitions
                # always read the last branch output (l.555-564)
                cur = y_list[-1]
                for j, seq in enumerate(t if isinstance(t[0], nn.Sequential) else [t]):
                    conv = seq[0]
                    hh, ww = _out_hw(conv, cur.H, cur.W)
                    ob = g.buffer(f"trans{si}.{i}.{j}", hh, ww, conv.out_channels)
                    g.conv(cur, conv, E.R(ob), act=A.ACT_LRELU, name=f"transition{si + 1}.{i}")
                    cur = E.R(ob)
                x_list.append(cur)
            last_stage = si == len(stages) - 1
            for mi, mod in enumerate(st):
                x_list = self._hr_module(g, mod, x_list, f"stage{si + 2}.{mi}", final=last_stage and
                                         mi == len(st) - 1)
            y_list = x_list
        return g

    def _bottleneck(self, g, blk, x, name):
        A = L
        H, W = x.H, x.W
        p = blk.conv1.out_channels
        a = g.buffer(name + ".a", H, W, p)
        g.conv(x, blk.conv1, E.R(a), act=A.ACT_LRELU, name=name + ".conv1")
        b = g.buffer(name + ".b", H, W, p)
        g.conv(E.R(a), blk.conv2, E.R(b), act=A.ACT_LRELU, name=name + ".conv2")
        if blk.downsample is not None:
            d = g.buffer(name + ".ds", H, W, blk.conv3.out_channels)
            g.conv(x, blk.downsample[0], E.R(d), name=name + ".downsample")
            res = E.R(d)
        else:
            res = x
        o = g.buffer(name + ".out", H, W, blk.conv3.out_channels)
        g.conv(E.R(b), blk.conv3, E.R(o), act=A.ACT_LRELU, res=res, name=name + ".conv3")
        return E.R(o)

    def _basic(self, g, blk, x, name):
        A = L
        h = g.buffer(name + ".h", x.H, x.W, blk.conv1.out_channels)
        g.conv(x, blk.conv1, E.R(h), act=A.ACT_LRELU, name=name + ".conv1")
        o = g.buffer(name + ".out", x.H, x.W, blk.conv2.out_channels)
        g.conv(E.R(h), blk.conv2, E.R(o), act=A.ACT_LRELU, res=x, name=name + ".conv2")
        return E.R(o)

    def _hr_module(self, g, mod, xs, name, final):
        """HighResolutionModule.forward (nets/HRNet.py:203-227) + (if final) the
        upsample/concat of nets/HRNet.py:576-582 writing into the 'cat' buffer."""
        A = L
        nbr = mod.num_branches
        xs = list(xs)
        for i in range(nbr):
            for k, blk in enumerate(mod.branches[i]):
                assert blk.downsample is None
                xs[i] = self._basic(g, blk, xs[i], f"{name}.branches.{i}.{k}")
        if nbr == 1:
            return xs
        H, W = xs[0].H, xs[0].W
        cat = None
        if final:
            last = sum(x.c for x in xs)
            cat = g.buffer("cat", H, W, last)
        ys = []
        for i in range(len(mod.fuse_layers)):
            ys.append(self._fuse_output(g, mod, xs, i, cat, final, name))
        if not final:
            return ys
        # final upsample of every branch into the concat buffer
        off = ys[0].c
        for i in range(1, len(ys)):
            g.fuse([ys[i]], E.R(cat, off, ys[i].c))
            off += ys[i].c
        self._heads(g, E.R(cat))
        return ys

    def _fuse_output(self, g, mod, xs, i, cat, final, name):
        """Fused output i of a HighResolutionModule (nets/HRNet.py:209-225): the sum of
        branch i and every other branch resized to it (1x1 conv + upsample from coarser
        branches, strided 3x3 chains from finer ones), LeakyReLU."""
        A = L
        nbr = len(xs)
        H, W = xs[0].H, xs[0].W
        fl = mod.fuse_layers[i]
        ups = []
        for j in range(i + 1, nbr):
            cv = fl[j][0]
            t = g.buffer(f"{name}.fuse.{i}.{j}", xs[j].H, xs[j].W, cv.out_channels)
            g.conv(xs[j], cv, E.R(t), name=f"{name}.fuse_layers.{i}.{j}")
            ups.append(E.R(t))
        if i == 0:
            out = E.R(cat, 0, xs[0].c) if final else E.R(g.buffer(f"{name}.y{i}", H, W, xs[0].c))
            self._fuse_many(g, [xs[0]] + ups, out, A.ACT_LRELU, f"{name}.pre{i}")
            return out
        base = xs[i]
        if ups:
            t = g.buffer(f"{name}.sum{i}", xs[i].H, xs[i].W, xs[i].c)
            self._fuse_many(g, [xs[i]] + ups, E.R(t), A.ACT_NONE, f"{name}.pre{i}")
            base = E.R(t)
        acc = base
        for j in range(i):
            seq = fl[j]
            cur = xs[j]
            for k in range(len(seq) - 1):
                cv = seq[k][0]
                hh, ww = _out_hw(cv, cur.H, cur.W)
                t = g.buffer(f"{name}.down.{i}.{j}.{k}", hh, ww, cv.out_channels)
                g.conv(cur, cv, E.R(t), act=A.ACT_LRELU, name=f"{name}.fuse_layers.{i}.{j}.{k}")
                cur = E.R(t)
            cv = seq[len(seq) - 1][0]
            lastj = j == i - 1
            t = g.buffer(f"{name}.y{i}" if lastj else f"{name}.acc{i}.{j}", xs[i].H, xs[i].W, xs[i].c)
            g.conv(cur, cv, E.R(t), act=A.ACT_LRELU if lastj else A.ACT_NONE, res=acc,
                   name=f"{name}.fuse_layers.{i}.{j}")
            acc = E.R(t)
        return acc

    def _fuse_many(self, g, srcs, out, act, name):
        """sum of up to N multi-resolution terms as chained 3-input fuse kernels."""
        while len(srcs) > 3:
            t = g.buffer(name + f".part{len(srcs)}", out.H, out.W, out.c)
            g.fuse(srcs[:3], E.R(t))
            srcs = [E.R(t)] + srcs[3:]
        g.fuse(srcs, out, act=act)

    # DVIE_FUSE_HEADS=0: the two 1x1 head convs as separate launches (A/B runs)
    fuse_heads = os.environ.get("DVIE_FUSE_HEADS", "1") != "0"
    _stack_limit = 0xFFFFFF00  # bytes of one image of the stacked hidden map (32-bit buffer range)

    def _heads(self, g, cat):
        """rgb_layer / seg_layer (nets/HRNet.py:410-442 of the reference).  Both start with a
        1x1 448 -> 448 conv + LeakyReLU over the same concat: run as one stacked 448 -> 896
        conv (E.StackedConv) whose halves feed the two 3x3 output convs."""
        A = L
        H, W = cat.H, cat.W
        last = cat.c
        if getattr(self, "_stacked_heads", None) is None:
            self._stacked_heads = E.StackedConv([self.rgb_layer[0], self.seg_layer[0]]) if self.fuse_heads else False
        st = self._stacked_heads
        # the 3x3 output convs address one image of the stacked buffer through a 32-bit
        # buffer range: keep the two hidden maps separate where 2x448 channels exceed it
        # (fp32 at 1024x2048)
        es = 2 if g.dtype == torch.bfloat16 else 4
        fits = H * W * 2 * last * es < self._stack_limit
        if st and fits and (getattr(g, "dry", False) or st.contiguous()):
            hh = g.buffer("heads_hidden", H, W, 2 * last)
            g.conv(cat, st, E.R(hh), act=A.ACT_LRELU, name="heads.0")
            hr, hs = E.R(hh, 0, last), E.R(hh, last, last)
        else:
            hr = E.R(g.buffer("rgb_hidden", H, W, last))
            g.conv(cat, self.rgb_layer[0], hr, act=A.ACT_LRELU, name="rgb_layer.0")
            hs = E.R(g.buffer("seg_hidden", H, W, last))
            g.conv(cat, self.seg_layer[0], hs, act=A.ACT_LRELU, name="seg_layer.0")
        rgb = g.buffer("rgb", H, W, E.rup(self.rgb_out_dim, 8), dtype=torch.float32, external=True)
        g.conv(hr, self.rgb_layer[2], E.R(rgb), name="rgb_layer.2")
        seg = g.buffer("segout", H, W, E.rup(self.seg_out_dim, 8), dtype=torch.float32, external=True)
        g.conv(hs, self.seg_layer[2], E.R(seg), name="seg_layer.2")
        g.output("rgb", E.R(rgb), self.rgb_out_dim)
        g.output("segout", E.R(seg), self.seg_out_dim)

    def _build_plan(self, key):
        n, H, W, dtype, train, dev, xgrad, export = key
        self._export_stem = export
        try:
            g = self._lower(E.Graph(dtype), H, W, xgrad=xgrad, vgrad=bool(train))
        finally:
            self._export_stem = False
        return g.compile(n, dev, backward=train)

    # set by InterRefineNet / InterStage3Net: every forward also writes the detached stem
    # features [frames (3F), seg_encoder(seg_k) (4 each)] to `last_stem` (B, 7F, H, W)
    export_stem = False
    last_stem = None

    def _on_moved(self):
        self._pool.clear()

    # ---- execution ----
    def run_forward(self, inputs, train):
        x, seg = inputs[:2]
        n, _, H, W = x.shape
        L.require_gpu(x)
        xgrad = bool(train) and bool(getattr(self, "_in_needs", (False,))[0])
        plan = self._pool.acquire((n, H, W, self.dtype, bool(train), x.device, xgrad, bool(self.export_stem)))
        xs, ss = getattr(self, "_parts", (None, None))
        if xs is not None:
            plan.set_input_parts("x", xs)
        else:
            plan.set_input("x", x)
        if ss is not None:
            plan.set_input_parts("seg", ss)
        else:
            plan.set_input("seg", seg)
        if self.export_stem:
            F = self.n_frames
            stem = torch.empty((n, 7 * F, H, W), dtype=torch.float32, device=x.device)
            plan.set_output_nchw("stem_x", stem[:, :3 * F])
            for k in range(F):
                plan.set_output_nchw(f"stem_seg{k}", stem[:, 3 * F + 4 * k:3 * F + 4 * k + 4])
            self.last_stem = stem
        if len(inputs) > 2:
            plan.set_input("vae", inputs[2])
        rgb = torch.empty((n, H, W, E.rup(self.rgb_out_dim, 8)), dtype=torch.float32, device=x.device)
        segout = torch.empty((n, H, W, E.rup(self.seg_out_dim, 8)), dtype=torch.float32, device=x.device)
        plan.set_output("rgb", rgb)
        plan.set_output("segout", segout)
        plan.run_forward()
        self.last_plan = plan
        return plan, (rgb.permute(0, 3, 1, 2)[:, :self.rgb_out_dim], segout.permute(0, 3, 1, 2)[:, :self.seg_out_dim])

    # set by runners.comm.GradSync: (bucket_bytes, fn(lo, hi)) called as soon as the flat
    # gradient range [lo, hi) is final during the backward pass
    grad_hook = None

    def _buckets(self, plan, bucket_bytes):
        key = ("buckets", bucket_bytes)
        if key in plan.__dict__:
            return plan.__dict__[key]
        end = {}
        for p, (off, n, _) in zip(self._flat_params, self._flat_specs):
            end[id(p)] = off + n
        total = self._flat.numel()
        cuts, ranges, last, hi, done = [], [], 0, 0, 0
        for idx, lay in plan.completions:
            if isinstance(lay.m, E.StackedConv):
                ps = lay.m.params()
            else:
                ps = [lay.m.weight] + ([lay.m.bias] if lay.m.bias is not None else [])
            hi = max([hi] + [end[id(p)] for p in ps])
            done += sum(p.numel() for p in ps)
            # the flat layout comes from a dry lowering where the two 448-channel head convs
            # are one stacked layer ([rgb.w, seg.w, rgb.b, seg.b]); a plan that keeps them
            # separate (fp32 at 1024x2048, `fits` in _heads) completes them one by one, so a
            # prefix [0, hi) is final only once every parameter below hi has completed
            if done == hi and (hi - last) * 4 >= bucket_bytes and hi < total:
                cuts.append(idx)
                ranges.append((last, hi))
                last = hi
        assert done == total, "every parameter gradient must complete in the backward plan"
        ranges.append((last, total))
        plan.__dict__[key] = (cuts, ranges)
        return cuts, ranges

    def run_backward(self, plan, inputs, grads, needs):
        accumulate = self.grad_views(self._trunk_params())
        plan.set_param_grads(accumulate)
        g_rgb, g_seg = grads
        if E.DEBUG_NAN:
            print(f"[dvie nan] HRNet output grads finite: rgb {bool(torch.isfinite(g_rgb).all())} "
                  f"seg {bool(torch.isfinite(g_seg).all())}", flush=True)
        plan.set_output_grad("rgb", g_rgb.float())
        plan.set_output_grad("segout", g_seg.float())
        gx = gv = None
        if "x" in plan.ext_grad:
            gx = torch.empty(inputs[0].shape, dtype=torch.float32, device=inputs[0].device)
            plan.set_input_grad("x", gx)
        if "vae" in plan.ext_grad:
            gv = torch.empty(inputs[2].shape, dtype=torch.float32, device=inputs[2].device)
            plan.set_input_grad("vae", gv)
        hook = self.grad_hook
        if hook is None:
            plan.run_backward()
        else:
            cuts, ranges = self._buckets(plan, hook[0])
            plan.run_backward(cuts=cuts, on_cut=lambda k: hook[1](*ranges[k]))
            hook[1](*ranges[-1])
        return [gx, None] + ([gv] if len(inputs) > 2 else [])

    def forward_split(self, x, seg):
        """x: (B, 3F, H, W) frames in [-1, 1]; seg: (B, 20F, H, W) one-hot segmentations.
        Either may also be a list of the F per-frame tensors ((B, 3, H, W) / (B, 20, H, W),
        fp32, equal strides): the plan's input ops then read them in place, with no
        concatenation (frames that need a gradient are concatenated)."""
        xs = list(x) if isinstance(x, (list, tuple)) else None
        ss = list(seg) if isinstance(seg, (list, tuple)) else None
        def in_place(ts, grad_ok=False):
            return (all(t.dtype == torch.float32 and t.stride() == ts[0].stride() and t.shape == ts[0].shape
                        for t in ts) and (grad_ok or not any(t.requires_grad for t in ts)))

        if xs is not None and not in_place(xs):
            x, xs = torch.cat([t.float() for t in xs], 1), None
        if ss is not None and not in_place(ss, grad_ok=True):
            seg, ss = torch.cat([t.float() for t in ss], 1), None
        x = xs[0] if xs is not None else x.float()  # stands in for the frames (shape, device)
        seg = ss[0] if ss is not None else seg.float()
        self._parts = (xs, ss)
        try:
            return PlanFunction.apply(self, 2, x, seg, *self._flat_params)
        finally:
            self._parts = (None, None)

    def forward(self, input):
        F = self.n_frames
        if self.syn_type == "extra" and self.fix_init:
            x, seg = input[:, :9], input[:, 9:9 + 20 * F]
        else:
            x, seg = input[:, :3 * F], input[:, 3 * F:3 * F + 20 * F]
        rgb, seg_out = self.forward_split(x, seg)
        if self.syn_type == "extra" and self.inpaint_mask:
            mask = torch.sigmoid(rgb[:, 3 * self.npo:])
            return rgb[:, :3 * self.npo], seg_out, mask
        return rgb, seg_out
