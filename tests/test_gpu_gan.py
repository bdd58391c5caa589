"""GPU parity of the GAN side (InterGANNet): discriminator plans (HIP convs, BatchNorm with
batch statistics, head), channel softmax, fused Adam, and one InterGANTrainer step, against
the CPU oracle (oracle/disc.py, itself pinned to the reference by tests/golden/disc.npz).

Tolerances: fp32 scores 1e-4 relative; gradients by relative L2 (1e-3) because a
LeakyReLU input within rounding of zero may take the other branch; BatchNorm-preceding
conv biases have an exactly-zero true gradient and are compared absolutely.
"""
import os
import types

import numpy as np
import pytest
import torch

import inputs
from oracle import disc as OD
from oracle import hrnet as OH
from oracle import losses as OL
from oracle import step as OS

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(1e-30, float(b.norm())))


def make_disc(kind, seed, prec, dev):
    os.environ["DVIE_PRECISION"] = prec
    from deep_video_interpolation_extrapolation_amd import nets
    torch.manual_seed(seed)
    cls = nets.FrameDiscriminator if kind == "frame" else nets.VideoDiscriminator
    return cls(types.SimpleNamespace(seg_disc=True, precision=prec)).to(dev)


@pytest.mark.parametrize("kind,seed", [("frame", 31), ("video", 32)])
@pytest.mark.parametrize("hw", [(128, 128), (128, 256)])
def test_disc_fp32_matches_oracle(dev, kind, seed, hw):
    H, W = hw
    d = make_disc(kind, seed, "fp32", dev)
    spec = (OD.FRAME if kind == "frame" else OD.VIDEO)(23)
    P = OD.init_params(spec, seed)
    sd = d.state_dict()
    for k, v in P.items():  # seeded init identical to the reference construction order
        assert torch.equal(sd[k].cpu(), v), k
    x, seg, ix, iseg, gout = inputs.disc_inputs(2, H, W)
    ins = [x, seg] + ([ix, iseg] if kind == "video" else [])
    # HIP first: its LeakyReLU branch decisions are imposed on the fp64 oracle, so that
    # an activation within rounding of zero that takes the other branch in fp32 (a kink
    # flip; at the 8x8 level one flip moves every lower-layer gradient by ~1/sqrt(24k))
    # does not mask a real error.  Then the comparison is smooth and tight.
    gins = [v.to(dev).requires_grad_(True) for v in ins]
    got = d(*gins)
    got.backward(gout.to(dev))
    torch.cuda.synchronize()
    masks = d.activation_signs()

    def oracle(dt, masks=None):
        st = {k[:-len(".running_mean")]: (P[k].clone().to(dt), P[k[:-4] + "var"].clone().to(dt))
              for k in P if k.endswith("running_mean")}
        oi = [v.clone().to(dt).requires_grad_(True) for v in ins]
        pr = {k: v.clone().to(dt).requires_grad_(True) for k, v in P.items() if "running" not in k}
        r = OD.forward(pr, spec, torch.cat(oi, 1), training=True, stats=st, masks=masks)
        r.backward(gout.to(dt))
        return r, oi, pr, st

    ref, oins, params, stats = oracle(torch.float64, masks)
    e = rel_l2(got.detach(), ref.detach())
    assert e < 1e-5, e
    for a, b in zip(gins, oins):
        e = rel_l2(a.grad, b.grad)
        assert e < 2e-4, e
    named = dict(d.named_parameters())
    for k, v in params.items():
        if k.endswith(".bias") and k.replace("bias", "weight") in P and P[k.replace("bias", "weight")].dim() == 4 \
                and f"layer.{int(k.split('.')[1]) + 1}.running_mean" in P:
            assert float(named[k].grad.abs().max()) < 1e-4, k  # conv bias before BatchNorm: zero gradient
            continue
        e = rel_l2(named[k].grad, v.grad)
        assert e < 2e-4, (k, e)
    for name, (rm, rv) in stats.items():
        assert rel_l2(sd[name + ".running_mean"], rm) < 1e-4
        assert rel_l2(sd[name + ".running_var"], rv) < 1e-4
    assert int(sd[list(stats)[0] + ".num_batches_tracked"]) == 1


VARIANTS = [("FrameLocalDiscriminator", 51), ("FrameSNDiscriminator", 52), ("FrameSNLocalDiscriminator", 53),
            ("VideoLocalDiscriminator", 54), ("VideoSNDiscriminator", 55), ("VideoSNLocalDiscriminator", 56)]


@pytest.mark.parametrize("cls,seed", VARIANTS)
@pytest.mark.parametrize("uvgrad", [False, True])
def test_disc_variant_fp32_matches_oracle(dev, cls, seed, uvgrad):
    """Local (map output) and SpectralNorm discriminators (HIP power iteration + sigma
    adjoint, dvie_sn_fwd / dvie_sn_bwd) vs the fp64 oracle (itself pinned to G8) on the HIP
    run's LeakyReLU branches: output 1e-5, input / parameter gradients 2e-4 relative L2,
    u / v after the power iteration 1e-5.  uvgrad: u / v trainable (after set_net_grad(True))."""
    if uvgrad and "SN" not in cls:
        pytest.skip("no SpectralNorm")
    os.environ["DVIE_PRECISION"] = "fp32"
    from deep_video_interpolation_extrapolation_amd import nets
    from test_oracle_disc import run_variant
    torch.manual_seed(seed)
    d = nets.__dict__[cls](types.SimpleNamespace(seg_disc=True, precision="fp32")).to(dev)
    P = OD.init_params(OD.SPECS[cls](23), seed)
    sd = d.state_dict()
    assert set(P) <= set(sd)
    for k, v in P.items():
        assert torch.equal(sd[k].cpu(), v), k
    if uvgrad:
        for p in d.parameters():
            p.requires_grad = True
    x, seg, ix, iseg, gout = inputs.disc_inputs(2, 128, 128)
    ins = [x, seg] + ([ix, iseg] if cls.startswith("Video") else [])
    gins = [v.to(dev).requires_grad_(True) for v in ins]
    got = d(*gins)
    if got.dim() > 1:
        gout = inputs.disc_map_grad(tuple(got.shape))
    got.backward(gout.to(dev))
    torch.cuda.synchronize()
    ref, oins, params, _, _, _ = run_variant(cls, seed, uvgrad, torch.float64, masks=d.activation_signs())
    assert tuple(got.shape) == tuple(ref.shape)
    e = rel_l2(got.detach(), ref.detach())
    assert e < 1e-5, e
    for a, b in zip(gins, oins):
        e = rel_l2(a.grad, b.grad)
        assert e < 2e-4, e
    named = dict(d.named_parameters())
    sd = d.state_dict()
    for k, v in params.items():
        if k.endswith(("weight_u", "weight_v")):
            assert rel_l2(sd[k], v.detach()) < 1e-5, k
        if v.grad is None:
            assert named[k].grad is None, k
            continue
        if k.endswith(".bias") and f"layer.{int(k.split('.')[1]) + 1}.running_mean" in P:
            assert float(named[k].grad.abs().max()) < 1e-4, k  # conv bias before BatchNorm: zero gradient
            continue
        e = rel_l2(named[k].grad, v.grad)
        assert e < 2e-4, (k, e)


@pytest.mark.parametrize("kind,seed", [("frame", 31), ("video", 32)])
def test_disc_bf16_close_to_fp32(dev, kind, seed):
    x, seg, ix, iseg, gout = inputs.disc_inputs(2, 128, 256)
    ins = [v.to(dev) for v in ([x, seg] + ([ix, iseg] if kind == "video" else []))]
    a = make_disc(kind, seed, "fp32", dev)(*ins)
    b = make_disc(kind, seed, "bf16", dev)(*ins)
    torch.cuda.synchronize()
    assert torch.isfinite(b).all()
    assert rel_l2(b.detach(), a.detach()) < 5e-2, rel_l2(b.detach(), a.detach())


def test_channel_softmax_matches_torch(dev):
    from deep_video_interpolation_extrapolation_amd.nets import channel_softmax
    g = torch.Generator().manual_seed(4)
    x = torch.randn((2, 24, 16, 32), generator=g) * 3
    xs = x[:, 2:22]  # channel-strided view, as HRNet's NHWC output slice
    gy = torch.randn((2, 20, 16, 32), generator=g)
    xr = xs.clone().requires_grad_(True)
    yr = torch.softmax(xr, 1)
    yr.backward(gy)
    xd = x.to(dev).permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)[:, 2:22].detach().requires_grad_(True)
    yd = channel_softmax(xd)
    yd.backward(gy.to(dev))
    assert float((yd.detach().cpu() - yr.detach()).abs().max()) < 1e-6
    assert float((xd.grad.cpu() - xr.grad).abs().max()) < 1e-6


def test_adam_matches_torch101_form(dev):
    from deep_video_interpolation_extrapolation_amd.optim import Adam
    g = torch.Generator().manual_seed(3)
    shapes = [(64, 3, 3, 3), (64,)]
    p0 = [torch.randn(s, generator=g) for s in shapes]
    mine = [t.clone().to(dev).requires_grad_(True) for t in p0]
    opt = Adam(mine, lr=1e-3)
    P = {i: t.clone() for i, t in enumerate(p0)}
    st = None
    for it in range(3):
        grads = [torch.randn(s, generator=g) * 10 ** -it for s in shapes]
        for m, gg in zip(mine, grads):
            m.grad = gg.to(dev)
        opt.step()
        P, st = OD.adam_101(P, dict(enumerate(grads)), 1e-3, st)
    for i, m in enumerate(mine):
        assert float((m.detach().cpu() - P[i]).abs().max()) < 1e-6
    assert set(opt.state_dict()["state"][0].keys()) == {"step", "exp_avg", "exp_avg_sq"}


def test_intergan_step_matches_oracle(dev):
    """InterGANTrainer (HRNet + FrameDiscriminator + VideoDiscriminator, seg_disc) one fp32
    step at 128x128 vs oracle.step.gan_step: loss dict 1e-4 relative; post-update weight
    sums of squares 1e-4 relative (generator) / 1e-3 (discriminators, excluding the
    zero-gradient BatchNorm-preceding conv biases, which Adam moves by +-lr on noise)."""
    os.environ["DVIE_PRECISION"] = "fp32"
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterGANTrainer import InterGANTrainer
    args = default_args("INTER", syn_type="inter", model="InterGANNet", gan=True, train_coarse=True, frame_disc=True,
                        video_disc=True, train_frame_disc=True, train_video_disc=True, seg_disc=True,
                        batch_size=2, input_h=128, input_w=128, precision="fp32", synthetic=2, num_workers=0,
                        split="train")
    torch.manual_seed(1024)
    tr = InterGANTrainer(args)
    m = tr.model.module
    P = {k: v.detach().cpu().clone() for k, v in m.coarse_model.state_dict().items()}
    Pf = {k: v.detach().cpu().clone() for k, v in m.frame_disc_model.state_dict().items() if "running" not in k
          and "num_batches" not in k}
    Pv = {k: v.detach().cpu().clone() for k, v in m.video_disc_model.state_dict().items() if "running" not in k
          and "num_batches" not in k}

    def stats_of(mod):
        sd = mod.state_dict()
        return {k[:-len(".running_mean")]: (sd[k].cpu().clone(), sd[k[:-4] + "var"].cpu().clone())
                for k in sd if k.endswith("running_mean")}

    sf, sv = stats_of(m.frame_disc_model), stats_of(m.video_disc_model)
    data = inputs.step_batch(2, 128, 128)
    ld = tr.step(data)
    ref, new, newf, newv, _, grads = OS.gan_step(P, Pf, Pv, OL.synthetic_vgg19_state(), data, sf, sv)
    assert list(ld.keys()) == list(ref.keys()), (list(ld.keys()), list(ref.keys()))
    np.testing.assert_allclose([float(ld[k]) for k in ref], [ref[k] for k in ref], rtol=1e-4)

    # Gradients: per-tensor relative L2 vs the fp32 oracle, median < 1e-3, worst < 3e-2
    # (LeakyReLU kink flips, see test_disc_fp32_matches_oracle; BatchNorm-preceding conv
    # biases, whose true gradient is 0, excluded).  Post-update weights: the first Adamax /
    # Adam step moves each weight by ~lr*sign(grad), so a near-zero gradient element whose
    # sign differs moves one weight by 2*lr: gate on the fraction of such elements.
    bn_bias = {f"layer.{i}.bias" for i in (2, 5)}
    for mod, g_ref, w_ref, tag in ((m.coarse_model, grads["g"], new, "g"), (m.frame_disc_model, grads["f"], newf, "f"),
                                   (m.video_disc_model, grads["v"], newv, "v")):
        named = dict(mod.named_parameters())
        errs, moved, total = [], 0, 0
        for k, gr in g_ref.items():
            if tag != "g" and k in bn_bias:
                continue
            errs.append(rel_l2(named[k].grad, gr))
            dw = (named[k].detach().cpu().double() - w_ref[k].double()).abs()
            moved += int((dw > 1e-4).sum())
            total += dw.numel()
        assert float(np.median(errs)) < 1e-3 and max(errs) < 3e-2, (tag, float(np.median(errs)), max(errs))
        assert moved <= 1e-3 * total, (tag, moved, total)


def test_intergan_vae_sn_two_steps(dev):
    """The reference's InterGAN configuration: VAEHRNet coarse model (KLD term) with the SN
    frame / video discriminators at 128x128, two fp32 steps: the second runs with SpectralNorm
    u / v trainable after set_net_grad(True) (per-parameter Adam step counts); losses stay
    finite, the KLD term sits after the CE term as in the reference (InterGANTrainer.py:406-409)
    and u moves with the power iteration."""
    os.environ["DVIE_PRECISION"] = "fp32"
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterGANTrainer import InterGANTrainer
    args = default_args("INTER", syn_type="inter", model="InterGANNet", gan=True, train_coarse=True, frame_disc=True,
                        video_disc=True, train_frame_disc=True, train_video_disc=True, seg_disc=True,
                        coarse_model="VAEHRNet", vae=True, frame_disc_model="FrameSNDiscriminator",
                        video_disc_model="VideoSNDiscriminator", batch_size=2, input_h=128, input_w=128,
                        precision="fp32", synthetic=2, num_workers=0, split="train")
    torch.manual_seed(1024)
    tr = InterGANTrainer(args)
    m = tr.model.module
    sn0 = m.frame_disc_model.layer[0].module
    u0 = sn0.weight_u.detach().clone()
    data = inputs.step_batch(2, 128, 128)
    ld1 = tr.step(data)
    assert sn0.weight_u.requires_grad  # set_net_grad(True) after the G pass, as the reference
    ld2 = tr.step(data)
    torch.cuda.synchronize()
    keys = list(ld1.keys())
    assert keys.index("coarse_kld_loss") == keys.index("coarse_ce_loss") + 1, keys
    assert keys[-1] == "loss_all" and list(ld2.keys()) == keys
    for ld in (ld1, ld2):
        assert all(np.isfinite(float(v)) for v in ld.values()), ld
    assert not torch.equal(sn0.weight_u.detach(), u0)
    assert sn0.weight_u.grad is not None and bool(torch.isfinite(sn0.weight_u.grad).all())
