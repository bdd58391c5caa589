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


def _setup(monkeypatch, prec):
    """the interpreter as the plans' executor on the CPU"""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    from deep_video_interpolation_extrapolation_amd import engine as E
    monkeypatch.setenv("DVIE_PRECISION", prec)
    monkeypatch.setattr(L, "require_gpu", lambda t: None)
    monkeypatch.setattr(L, "stream_ptr", lambda *a: 0)
    mem = Memory(torch.device("cpu"))
    track(mem, monkeypatch.setattr)
    ex = Executor(mem)
    monkeypatch.setattr(E, "OP_HOOK", ex)
    return ex


def _run(monkeypatch, prec, H=32, W=64):
    from deep_video_interpolation_extrapolation_amd import nets
    ex = _setup(monkeypatch, prec)
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
    for k in (L.OP_PACK, L.OP_CONV, L.OP_WGRAD, L.OP_WREDUCE, L.OP_EW):
        assert ex.kinds.get(k, 0) > 0, k
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
