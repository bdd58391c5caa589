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
    """InterGANTrainer (HRNet coarse model + FrameDiscriminator + VideoDiscriminator, seg_disc:
    the build-defined form that runs at any size) one fp32 step at 128x128 vs
    oracle.step.gan_step: loss dict 1e-4 relative; every generator and discriminator gradient
    against the fp64 oracle on this step's activation branches (all six discriminator passes
    imposed) within 1e-4 relative L2, 3e-4 where the gradient comes back through the
    discriminators' train-mode BatchNorm (all discriminator tensors, the generator's through the
    G passes); post-update weights within 1e-4 except a 1e-3 fraction (first Adamax / Adam step:
    +-lr on the sign of a near-zero gradient)."""
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
    sf64 = {k: (a.clone(), b.clone()) for k, (a, b) in sf.items()}
    sv64 = {k: (a.clone(), b.clone()) for k, (a, b) in sv.items()}
    data = inputs.step_batch(2, 128, 128)
    m.frame_disc_model.plan_log, m.video_disc_model.plan_log = [], []
    ld = tr.step(data)
    torch.cuda.synchronize()
    fl = [p.activation_signs() for p in m.frame_disc_model.plan_log]
    vl = [p.activation_signs() for p in m.video_disc_model.plan_log]
    m.frame_disc_model.plan_log = m.video_disc_model.plan_log = None
    ref, new, newf, newv, _, _ = OS.gan_step(P, Pf, Pv, OL.synthetic_vgg19_state(), data, sf, sv)
    assert list(ld.keys()) == list(ref.keys()), (list(ld.keys()), list(ref.keys()))
    np.testing.assert_allclose([float(ld[k]) for k in ref], [ref[k] for k in ref], rtol=1e-4)
    _, _, _, _, _, g64 = OS.gan_step(P, Pf, Pv, OL.synthetic_vgg19_state(), data, sf64, sv64,
                                     masks=m.coarse_model.last_plan.activation_signs(),
                                     vmasks=tr.RGBLoss.vgg_loss.vgg_net.last_plan.activation_signs(),
                                     gf_masks=fl[2], gv_masks=vl[2], df_masks=(fl[0], fl[1]), dv_masks=(vl[0], vl[1]),
                                     dtype=torch.float64)
    # conv biases right before a train-mode BatchNorm: true gradient 0 (frame disc: layer.2;
    # video disc: layers 2 and 5, oracle/disc.py FRAME / VIDEO)
    bn_bias = {"f": {"layer.2.bias"}, "v": {"layer.2.bias", "layer.5.bias"}}
    moved = total = 0
    for mod, g_ref, w_ref, tag in ((m.coarse_model, g64["g"], new, "g"), (m.frame_disc_model, g64["f"], newf, "f"),
                                   (m.video_disc_model, g64["v"], newv, "v")):
        named = dict(mod.named_parameters())
        errs = {}
        for k, gr in g_ref.items():
            if k in bn_bias.get(tag, ()):  # rounding noise, relative to the layer's weight gradient
                assert float(named[k].grad.norm()) <= 1e-3 * float(named[k[:-4] + "weight"].grad.norm()), k
                continue
            errs[k] = rel_l2(named[k].grad, gr)
            dw = (named[k].detach().cpu().double() - w_ref[k].double()).abs()
            moved += int((dw > 1e-4).sum())
            total += dw.numel()
        worst = max(errs, key=errs.get)
        print(f"{tag}: {len(errs)} gradients vs fp64 oracle on the same branches: relative L2 median "
              f"{np.median(list(errs.values())):.2e}, worst {errs[worst]:.2e} ({worst})")
        assert errs[worst] <= 3e-4, (tag, worst, errs[worst])
    assert moved <= 1e-3 * total, (moved, total)


def _uv(k):
    return k.endswith(("weight_u", "weight_v"))


def _disc_oracle_params(mod, cls):
    """the oracle's parameter set of a discriminator (u, v, weight_bar, bias; no running
    statistics, no SpectralNorm effective-weight scratch) from the module's state"""
    keys = set(OD.init_params(OD.SPECS[cls](23), 0))
    sd = mod.state_dict()
    return {k: sd[k].detach().cpu().clone() for k in keys if "running" not in k}


def _opt_state(opt, named, kind):
    """torch-format optimizer state -> oracle state (name -> dict); parameters without state
    (SpectralNorm u / v before their first gradient) are absent"""
    ids = {id(p): n for n, p in named.items()}
    out = {}
    for p, st in opt.state.items():
        if id(p) not in ids or "step" not in st:
            continue
        step = int(float(st["step"]))
        if kind == "adamax":
            out[ids[id(p)]] = dict(step=step, exp_avg=st["exp_avg"].detach().cpu().clone(),
                                   exp_inf=st["exp_inf"].detach().cpu().clone())
        else:
            out[ids[id(p)]] = dict(step=step, m=st["exp_avg"].detach().cpu().clone(),
                                   v=st["exp_avg_sq"].detach().cpu().clone())
    return out


def _vae_zero_bias(sd_keys):
    """VAE conv biases followed by train-mode BatchNorm (true gradient 0)"""
    out = set()
    for k in sd_keys:
        if k.startswith("vae_") and k.endswith(".bias"):
            pre, i = k[:-len(".bias")].rsplit(".", 1)
            if f"{pre}.{int(i) + 1}.running_mean" in sd_keys:
                out.add(k)
    return out


def test_intergan_vae_sn_steps_match_oracle(dev):
    """The reference's own InterGAN configuration (VAEHRNet coarse model with the
    KLD term, FrameSN / VideoSN discriminators, seg_disc, 128x128; InterGANNet.py:28-117,
    InterGANTrainer.py:376-456, KLD losses.py:50-60, SpectralNorm.py:14-67) for two fp32 steps
    against oracle.step.gan_step (pinned to the reference by G14, tests/test_oracle_gan.py).
    Step 2 starts from this implementation's post-step-1 state (weights, u / v, BatchNorm
    running statistics, optimizer states) with u / v trainable (set_net_grad(True)).  Per step:
    * loss dict (KLD after CE, as the reference) within 1e-4 relative of the fp32 oracle;
    * every gradient tensor -- generator (VAE encoder / decoder, mu / logvar FCs, HRNet trunk),
      both discriminators, and the u / v gradients of step 2 -- against the fp64 oracle evaluated
      on this step's activation branches (every LeakyReLU of every pass imposed): relative L2
      <= 1e-4, <= 3e-4 for the VAE encoder / decoder / FC tensors (their gradient comes back
      through train-mode BatchNorm backward, cancelling in fp32); BatchNorm-preceding conv
      biases (true gradient 0) at rounding level of their layer's weight gradient;
    * post-step weights within 1e-4 of the fp32 oracle's except a <= 1e-3 fraction (a first
      Adam / Adamax step moves a weight by +-lr on the sign of a near-zero gradient), u / v
      within 1e-5, running statistics within 1e-4."""
    os.environ["DVIE_PRECISION"] = "fp32"
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterGANTrainer import InterGANTrainer
    from oracle import vaehrnet as V
    FR, VI = "FrameSNDiscriminator", "VideoSNDiscriminator"
    args = default_args("INTER", syn_type="inter", model="InterGANNet", gan=True, train_coarse=True, frame_disc=True,
                        video_disc=True, train_frame_disc=True, train_video_disc=True, seg_disc=True,
                        coarse_model="VAEHRNet", vae=True, frame_disc_model=FR, video_disc_model=VI, batch_size=2,
                        input_h=128, input_w=128, precision="fp32", synthetic=2, num_workers=0, split="train")
    torch.manual_seed(1024)
    tr = InterGANTrainer(args)
    m = tr.model.module
    cm, fd, vd = m.coarse_model, m.frame_disc_model, m.video_disc_model
    named = {"g": dict(cm.named_parameters()), "f": dict(fd.named_parameters()), "v": dict(vd.named_parameters())}
    zero_b = _vae_zero_bias(set(cm.state_dict()))
    data = inputs.step_batch(2, 128, 128)
    vgg = OL.synthetic_vgg19_state()
    state = None
    for k in range(2):
        Pg = {n: p.detach().cpu().clone() for n, p in named["g"].items()}
        Pf, Pv = _disc_oracle_params(fd, FR), _disc_oracle_params(vd, VI)
        vst = V.bn_stats({n: t.detach().cpu().clone() for n, t in cm.state_dict().items()})
        if k > 0:
            state = {"g": _opt_state(tr.coarse_opt, named["g"], "adamax"),
                     "f": _opt_state(tr.frame_disc_opt, named["f"], "adam"),
                     "v": _opt_state(tr.video_disc_opt, named["v"], "adam")}
        fd.plan_log, vd.plan_log = [], []
        ld = tr.step(data)
        torch.cuda.synchronize()
        assert all(p.requires_grad for p in fd.parameters())  # set_net_grad(True) after the G pass
        eps = cm.last_eps.detach().cpu().clone()
        masks = dict(cm.last_plan.activation_signs())
        for r in (cm._enc, cm._dec):
            masks.update(r.last_plan.activation_signs())
        vmasks = tr.RGBLoss.vgg_loss.vgg_net.last_plan.activation_signs()
        fl = [p.activation_signs() for p in fd.plan_log]
        vl = [p.activation_signs() for p in vd.plan_log]
        fd.plan_log = vd.plan_log = None
        assert len(fl) == 3 and len(vl) == 3  # D(fake.detach()), D(real), frozen D(fake)
        kw = dict(frame_spec=FR, video_spec=VI, uv_grad=k > 0)
        ref, new, newf, newv, st32, _ = OS.gan_step(
            Pg, Pf, Pv, vgg, data, {}, {}, vae={"eps": eps, "stats": {n: (a.clone(), b.clone()) for n, (a, b) in
                                                                      vst.items()}},
            state=None if state is None else {t: {n: dict(d) for n, d in s.items()} for t, s in state.items()}, **kw)
        keys = list(ld.keys())
        assert keys == list(ref.keys()), (keys, list(ref.keys()))
        assert keys.index("coarse_kld_loss") == keys.index("coarse_ce_loss") + 1
        np.testing.assert_allclose([float(ld[n]) for n in ref], [ref[n] for n in ref], rtol=1e-4)
        _, _, _, _, _, g64 = OS.gan_step(
            Pg, Pf, Pv, vgg, data, {}, {}, vae={"eps": eps, "stats": vst}, masks=masks, vmasks=vmasks,
            gf_masks=fl[2], gv_masks=vl[2], df_masks=(fl[0], fl[1]), dv_masks=(vl[0], vl[1]),
            dtype=torch.float64, **kw)
        for tag in ("g", "f", "v"):
            errs = {}
            for n, gr in g64[tag].items():
                got = named[tag][n].grad
                assert got is not None, (k, tag, n)
                if n in zero_b:
                    w = named[tag][n[:-4] + "weight"].grad.double().norm()
                    assert float(got.double().norm()) <= 1e-3 * float(w), (k, n)
                    continue
                errs[n] = rel_l2(got, gr)
            if k == 0:  # u / v: no gradient in step 1 (requires_grad False until set_net_grad(True))
                assert all(named[tag][n].grad is None for n in named[tag] if _uv(n)), tag
            worst = max(errs, key=errs.get)
            print(f"step {k + 1} {tag}: {len(errs)} gradients vs fp64 oracle on the same branches: relative L2 "
                  f"median {np.median(list(errs.values())):.2e}, worst {errs[worst]:.2e} ({worst})")
            for n, e in errs.items():
                assert e <= (3e-4 if n.startswith(("vae_", "mu_fc", "logvar_fc")) else 1e-4), (k, tag, n, e)
        if k > 0:
            assert any(_uv(n) for n in g64["f"]) and any(_uv(n) for n in g64["v"])
        moved = total = 0
        for tag, ref_p in (("g", new), ("f", newf), ("v", newv)):
            sd = {"g": cm, "f": fd, "v": vd}[tag].state_dict()
            for n, w in ref_p.items():
                if n in zero_b:
                    continue
                got = sd[n].detach().cpu().double()
                if _uv(n):
                    assert rel_l2(got, w) < 1e-5, (k, n)
                    continue
                d = (got - w.double()).abs()
                moved += int((d > 1e-4).sum())
                total += d.numel()
        assert moved <= 1e-3 * total, (k, moved, total)
        sd = cm.state_dict()
        for n, (rm, rv) in st32["stats"][2].items():
            pre, i = n.rsplit(".", 1)
            assert rel_l2(sd[n + ".running_var"], rv) < 1e-4, (k, n)
            if k > 0 and f"{pre}.{int(i) - 1}.bias" in zero_b:
                continue  # the running mean carries step 1's +-lr noise move of the preceding conv bias
            assert rel_l2(sd[n + ".running_mean"], rm) < 1e-4, (k, n)
