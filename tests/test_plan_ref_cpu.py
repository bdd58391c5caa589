"""CPU: pin the descriptor interpreter of the layer-local GPU parity test (tests/plan_ref.py)
to the fp64 oracle.  The interpreter runs as the executor of a whole HRNet plan (engine.OP_HOOK:
every pack / conv / weight-gradient / reduction / pointwise descriptor of the forward and the
backward evaluated from its include/dvie.h meaning, nothing launched), and the plan's outputs
and parameter gradients must then equal the oracle's (oracle/hrnet.py, itself pinned to the
reference by G1).  So a descriptor the interpreter misreads would show here, on the CPU,
before the GPU test uses the interpreter as its reference."""
import types

import numpy as np
import torch

import inputs
from oracle import hrnet as O
from plan_ref import Executor, Memory, rel_l2, track


def _setup(monkeypatch, prec, ex_cls=None):
    """the interpreter as the plans' executor on the CPU"""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    from deep_video_interpolation_extrapolation_amd import engine as E
    monkeypatch.setenv("DVIE_PRECISION", prec)
    monkeypatch.setattr(L, "require_gpu", lambda t: None)
    monkeypatch.setattr(L, "stream_ptr", lambda *a: 0)
    mem = Memory(torch.device("cpu"))
    track(mem, monkeypatch.setattr)
    ex = (ex_cls or Executor)(mem)
    monkeypatch.setattr(E, "OP_HOOK", ex)
    return ex


def _run(monkeypatch, prec, H=32, W=64, ex_cls=None):
    from deep_video_interpolation_extrapolation_amd import nets
    ex = _setup(monkeypatch, prec, ex_cls)
    torch.manual_seed(1024)
    m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet"))
    x, seg = inputs.hrnet_input(2, H, W)
    g = torch.Generator().manual_seed(5)
    w1, w2 = torch.randn((2, 3, H, W), generator=g), torch.randn((2, 20, H, W), generator=g)
    rgb, s = m(x, seg)
    ((rgb * w1).sum() + (s * w2).sum()).backward()
    return m, x, seg, w1, w2, rgb.detach(), s.detach(), ex


def _oracle(m, x, seg, w1, w2, masks):
    P = {k: v.double().clone().requires_grad_(True) for k, v in O.init_params(1024).items()}
    rr, sr = O.forward(P, torch.cat([x, seg], 1).double(), masks=masks)
    ((rr * w1.double()).sum() + (sr * w2.double()).sum()).backward()
    return rr.detach(), sr.detach(), P


def test_interpreter_runs_the_fp32_hrnet_plan_like_the_oracle(monkeypatch):
    from deep_video_interpolation_extrapolation_amd import _lib as L
    m, x, seg, w1, w2, rgb, s, ex = _run(monkeypatch, "fp32")
    for k in (L.OP_PACK, L.OP_CONV, L.OP_WGRAD, L.OP_EW):
        assert ex.kinds.get(k, 0) > 0, k
    assert ex.kinds.get(L.OP_WREDUCE, 0) + ex.kinds.get(L.OP_WREDUCE_MULTI, 0) > 0
    masks = m.coarse_model.last_plan.activation_signs()
    rr, sr, P = _oracle(m, x, seg, w1, w2, masks)
    assert float((rgb.double() - rr).abs().max()) < 1e-5
    assert float((s.double() - sr).abs().max()) < 1e-5
    named = dict(m.coarse_model.named_parameters())
    errs = {k: rel_l2(named[k].grad, P[k].grad) for k in P}
    worst = max(errs, key=errs.get)
    print(f"interpreter vs oracle gradients: median {np.median(list(errs.values())):.2e}, worst {errs[worst]:.2e} "
          f"({worst})")
    assert errs[worst] <= 1e-5, (worst, errs[worst])


def test_interpreter_runs_the_bf16_hrnet_plan(monkeypatch):
    """bf16 plan: the fused head backward and seg-encoder backward descriptors
    (OP_HEAD3_BWD / OP_SEGENC_BWD) and the bf16 storage path of the interpreter; results
    within bf16 distance of the fp64 oracle."""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    m, x, seg, w1, w2, rgb, s, ex = _run(monkeypatch, "bf16")
    assert ex.kinds.get(L.OP_HEAD3_BWD, 0) == 1 and ex.kinds.get(L.OP_SEGENC_BWD, 0) == 2
    masks = m.coarse_model.last_plan.activation_signs()
    rr, sr, P = _oracle(m, x, seg, w1, w2, masks)
    assert rel_l2(rgb, rr) < 2e-2 and rel_l2(s, sr) < 2e-2
    named = dict(m.coarse_model.named_parameters())
    errs = {k: rel_l2(named[k].grad, P[k].grad) for k in P}
    worst = max(errs, key=errs.get)
    print(f"bf16 interpreter vs oracle gradients: median {np.median(list(errs.values())):.2e}, worst "
          f"{errs[worst]:.2e} ({worst})")
    assert float(np.median(list(errs.values()))) < 2e-2


def test_interpreter_runs_the_vgg_loss_plan(monkeypatch):
    """The VGG19 perceptual-loss plan (reference losses.py:157-180): the normalising input
    ops, ReLU convs, 2x2 average pools, the feature-L1 loss ops and their backward (L1 sign,
    pool adjoints, data gradients, the NCHW gradient pack through the normalisation)."""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    from deep_video_interpolation_extrapolation_amd.losses import VGGLoss
    from oracle import losses as OL
    ex = _setup(monkeypatch, "fp32")
    vl = VGGLoss()
    g = torch.Generator().manual_seed(11)
    a = (torch.rand((2, 3, 32, 64), generator=g) * 2 - 1).requires_grad_(True)
    b = torch.rand((2, 3, 32, 64), generator=g) * 2 - 1
    loss = vl(a, b, normed=False)
    loss.backward()
    for k in (L.OP_PACK, L.OP_CONV, L.OP_EW, L.OP_LOSS):
        assert ex.kinds.get(k, 0) > 0, k
    masks = vl.vgg_net.last_plan.activation_signs()
    state = {k: v.double() for k, v in OL.synthetic_vgg19_state().items()}
    ad = a.detach().double().requires_grad_(True)
    ref = OL.vgg_loss(state, ad, b.double(), normed=False, masks=masks)
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-6 * abs(float(ref))
    e = rel_l2(a.grad, ad.grad)
    print(f"VGG loss plan: value {float(loss):.6f} vs {float(ref):.6f}, input gradient rel L2 {e:.2e}")
    assert e <= 1e-5


class _FusedBwdCheck(Executor):
    """The interpreter as executor, plus an INDEPENDENT float64 evaluation of the two
    descriptors only the bf16 plan emits (OP_HEAD3_BWD, OP_SEGENC_BWD): torch autograd's
    conv2d input / weight gradients over the OIHW parameters (reference nets/HRNet.py:
    rgb_layer l.410-442, seg_encoder l.358-364), on the very bf16 operands the descriptor
    reads.  It shares nothing with the interpreter's packed-weight / tap-order arithmetic, so a
    misread tap flip or channel map in either descriptor shows as a per-tensor mismatch."""

    def __init__(self, mem):
        super().__init__(mem)
        self.expect = {}  # parameter name -> float64 gradient (summed over the descriptors)
        self.dh = []  # (written dh view, float64 expectation)

    def _nchw(self, ptr, n, h, w, ld, c):
        from plan_ref import nhwc
        return self.mem.view(ptr, *nhwc(n, h, w, ld, c), torch.bfloat16).double().permute(0, 3, 1, 2)

    def _add(self, name, v):
        self.expect[name] = self.expect.get(name, 0) + v

    def _unpack(self, lay, xp):
        """packed input channels -> the layer's source channels (its cmap)"""
        x = torch.zeros((xp.shape[0], lay.cin) + tuple(xp.shape[2:]), dtype=xp.dtype)
        for j, ci in enumerate(lay.cmap):
            if 0 <= ci < lay.cin:
                x[:, ci] = xp[:, j]
        return x

    def __call__(self, plan, arr, i, meta, run):
        from deep_video_interpolation_extrapolation_amd import _lib as L
        from torch.nn.grad import conv2d_input, conv2d_weight
        o = arr[i]
        lays = {lay.name: lay for lay in plan.g.layers}
        post = None
        if o.kind == L.OP_HEAD3_BWD:
            d = o.u.head3
            lay = lays[meta["name"].split("+")[0]]
            W = lay.m.weight.detach().to(torch.bfloat16).double()
            pad = lay.m.padding
            hp = self._nchw(d.h, d.n, d.hgt, d.wid, d.h_ld, d.c)
            h = self._unpack(lay, hp)
            g = self._nchw(d.g, d.n, d.hgt, d.wid, d.g_ld, d.cout)[:, :lay.cout]
            self._add(lay.name + ".weight", conv2d_weight(h, W.shape, g, padding=pad))
            dx = conv2d_input(h.shape, W, g, padding=pad)
            dhp = torch.zeros_like(hp)
            for j, ci in enumerate(lay.cmap):
                if 0 <= ci < lay.cin:
                    dhp[:, j] = dx[:, ci]
            if d.dact:  # LeakyReLU derivative from the stored activation's sign
                dhp = dhp * torch.where(hp > 0, 1.0, d.alpha)
            post = (d, dhp.permute(0, 2, 3, 1))
        elif o.kind == L.OP_SEGENC_BWD:
            d = o.u.segenc_bwd
            n, h, w = d.n, d.h, d.w
            l0, l2, l4 = lays["seg_encoder.0"], lays["seg_encoder.2"], lays["seg_encoder.4"]
            W4 = l4.m.weight.detach().to(torch.bfloat16).double()
            W2 = l2.m.weight.detach().to(torch.bfloat16).double()
            e2 = self._nchw(d.e2, n, h, w, d.e2_ld, 32)
            e1 = self._nchw(d.e1, n, h, w, d.e1_ld, 32)
            inp = self._unpack(l0, self._nchw(d.inp, n, h, w, d.in_ld, l0.cin_p))
            dout = self._nchw(d.dout, n, h, w, d.dout_ld, 8)[:, :l4.cout]

            def elu_d(e):  # ELU(1)' from its output value
                return torch.where(e > 0, 1.0, e + 1.0)

            def bf(v):  # d_e2 / d_e1 are rounded to bf16 on chip
                return v.to(torch.bfloat16).double()

            de2 = bf(conv2d_input(e2.shape, W4, dout, padding=1) * elu_d(e2))
            de1 = bf(conv2d_input(e1.shape, W2, de2, padding=1) * elu_d(e1))
            for lay, x, gg in ((l4, e2, dout), (l2, e1, de2), (l0, inp, de1)):
                self._add(lay.name + ".weight", conv2d_weight(x, lay.m.weight.shape, gg, padding=1))
                self._add(lay.name + ".bias", gg.sum((0, 2, 3)))
        super().__call__(plan, arr, i, meta, run)
        if post is not None:
            d, v = post
            self.dh.append((self.mem.view(d.dh, *__import__("plan_ref").nhwc(d.n, d.hgt, d.wid, d.dh_ld, d.c),
                                          torch.bfloat16).double(), v))


def test_bf16_fused_backward_descriptors_per_tensor(monkeypatch):
    """Verdict r05 item 7: the parameter gradients the bf16-only fused descriptors produce
    (rgb_layer.2 through OP_HEAD3_BWD; seg_encoder.0/2/4 through two OP_SEGENC_BWD, one per
    segmentation map, summed by their slab reductions) each gated PER TENSOR against the
    independent float64 autograd evaluation above, at <= 1e-5 relative L2 (fp32 slab sums of
    float64 products), and the head's data gradient at the bf16 output-rounding bar."""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    m, x, seg, w1, w2, rgb, s, ex = _run(monkeypatch, "bf16", ex_cls=_FusedBwdCheck)
    assert ex.kinds.get(L.OP_HEAD3_BWD, 0) == 1 and ex.kinds.get(L.OP_SEGENC_BWD, 0) == 2
    named = dict(m.coarse_model.named_parameters())
    want = {"rgb_layer.2.weight"} | {f"seg_encoder.{k}.{p}" for k in (0, 2, 4) for p in ("weight", "bias")}
    assert want <= set(ex.expect), sorted(ex.expect)
    # the head's bias gradient comes from its own column-sum op (interpreted generically)
    errs = {k: rel_l2(named[k].grad, ex.expect[k]) for k in sorted(ex.expect)}
    for k, e in errs.items():
        print(f"  {k:24s} rel L2 {e:.2e}")
    bad = {k: e for k, e in errs.items() if not e <= 1e-5}
    assert not bad, bad
    assert len(ex.dh) == 1
    got, ref = ex.dh[0]
    e = rel_l2(got, ref)
    print(f"  rgb_layer.2 dh (bf16)     rel L2 {e:.2e}")
    assert e <= 4e-3


def test_stride2_one_launch_lowerings_equal_the_per_phase_forms(monkeypatch):
    """The stride-2 lowerings of the bf16 plan -- the data gradient as ONE phase-split launch
    (dvie_conv_desc.phc) and the weight gradient as four phase-view launches into one shared
    9-tap slab set (dvie_wgrad_desc.ws_taps / tmap) -- give the same parameter and input
    gradients as the per-phase / per-tap forms they replace (DVIE_PH4=0, DVIE_WGRAD_S2=0),
    with the interpreter as executor.  32 x 256 so that every stride-2 layer's output width
    is a multiple of 64 (the phase-view condition) and both lowerings are taken (DVIE_WGRAD_S2=2:
    every eligible layer, not only the >= 256-channel inputs of the default)."""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    res = {}
    for tag, env in (("new", {"DVIE_WGRAD_S2": "2"}), ("old", {"DVIE_PH4": "0", "DVIE_WGRAD_S2": "0"})):
        with monkeypatch.context() as mp:
            for k, v in env.items():
                mp.setenv(k, v)
            m, x, seg, w1, w2, rgb, s, ex = _run(mp, "bf16", H=32, W=256)
            plan = m.coarse_model.last_plan
            n_ph = sum(1 for o in plan.bwd if o.kind == L.OP_CONV and o.u.conv.phc)
            n_ws = sum(1 for o in plan.bwd if o.kind == L.OP_WGRAD and o.u.wgrad.ws_taps)
            res[tag] = ({k: p.grad.clone() for k, p in m.coarse_model.named_parameters()}, n_ph, n_ws)
    g_new, n_ph, n_ws = res["new"]
    g_old, n_ph0, n_ws0 = res["old"]
    print(f"one-launch stride-2 data gradients {n_ph}, phase-view weight-gradient launches {n_ws}")
    assert n_ph0 == 0 and n_ws0 == 0
    assert n_ph == 6 and n_ws == 4 * 7, (n_ph, n_ws)  # transition1.1 (256 channels) keeps four phase launches
    errs = {k: rel_l2(g_new[k], g_old[k]) for k in g_old}
    worst = max(errs, key=errs.get)
    print(f"worst {errs[worst]:.2e} ({worst})")
    assert errs[worst] <= 1e-6, (worst, errs[worst])
