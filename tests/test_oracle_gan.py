"""The oracle's InterGAN step (oracle.step.gan_step with a VAEHRNet coarse model, KLD and the
SpectralNorm frame / video discriminators) against G14 (tests/golden/gan_vae.npz): two steps of
the reference's own runnable InterGAN configuration (nets/InterGANNet.py:28-117 with
nets/HRNet.py:702-1061 VAEHRNet, nets/FrameDisc.py / nets/VidDisc.py SN variants,
nets/SpectralNorm.py:14-67; runners/InterGANTrainer.py:376-456, KLD losses.py:50-60), 128x128,
batch 2.  Step 2 runs with u / v trainable (set_net_grad(True) after step 1).  CPU only.
The fixture's torch.optim.Adam is this container's (eps after the bias correction), so the
discriminator updates are checked with oracle.disc.adam_torch2 here; the reference's torch
1.0.1 form (adam_101, what the product runs) differs from it only through eps and is pinned by
test_oracle_disc.test_adam_101_matches_torch_adam_at_zero_eps."""
import os

import numpy as np
import torch

import inputs
from oracle import disc as OD
from oracle import losses as OL
from oracle import step as OS
from oracle import vaehrnet as V

G = os.path.join(os.path.dirname(__file__), "golden")
FRAME, VIDEO = "FrameSNDiscriminator", "VideoSNDiscriminator"


def reference_init():
    """VAEHRNet, then the frame and video SN discriminators on one RNG stream (the
    InterGANNet construction order, nets/InterGANNet.py:8-19), seed 1024."""
    g = V.init_params(1024)
    f = OD.init_params(OD.SPECS[FRAME](23), None)
    v = OD.init_params(OD.SPECS[VIDEO](23), None)
    return g, f, v


def _params(sd):
    return {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}


def _bn_biases(sd):
    """conv biases followed by a train-mode BatchNorm: their true gradient is exactly 0 (the
    batch mean cancels them), so both sides hold rounding noise there"""
    out = set()
    for k in sd:
        if k.endswith(".bias") and "." in k[:-len(".bias")]:
            pre, i = k[:-len(".bias")].rsplit(".", 1)
            if i.isdigit() and f"{pre}.{int(i) + 1}.running_mean" in sd:
                out.add(k)
    return out


def _check_sumsq(got, names, ref, rtol, tag, zero=()):
    keep = [i for i, n in enumerate(names) if str(n) not in zero]
    for i, n in enumerate(names):
        if str(n) in zero:  # rounding level on both sides, relative to the layer's weight gradient
            w2 = float((got[str(n)[:-4] + "weight"].double() ** 2).sum())
            assert float((got[str(n)].double() ** 2).sum()) < 1e-6 * w2 and ref[i, 1] < 1e-6 * w2, (tag, str(n))
    names, ref = names[keep], ref[keep]
    g2 = np.array([float((got[str(n)].double() ** 2).sum()) for n in names])
    rel = np.abs(g2 - ref[:, 1]) / np.maximum(np.abs(ref[:, 1]), 1e-30)
    assert float(np.median(rel)) < rtol[0] and float(rel.max()) < rtol[1], (tag, float(np.median(rel)),
                                                                           str(names[int(rel.argmax())]),
                                                                           float(rel.max()))


def test_gan_vae_sn_two_steps_match_reference(monkeypatch):
    # G14 ran under this container's torch, whose backward of a SpectralNorm call sees the u / v
    # a later call of the same step wrote (torch 1.0.1 saved each call's own): generate the
    # oracle side with that semantics here; oracle.disc.SN_PER_CALL (1.0.1, the product's) is
    # the same code with per-call copies
    monkeypatch.setattr(OD, "SN_PER_CALL", False)
    f = np.load(os.path.join(G, "gan_vae.npz"))
    sg, sf, sv = reference_init()
    for sd, tag in ((sg, "g"), (sf, "f"), (sv, "v")):
        names = [str(n) for n in f[tag + "_init_names"]]
        assert {n for n in names if "num_batches" not in n} == set(sd), tag
        ref = f[tag + "_init"]
        for i, n in enumerate(names):
            if n in sd:
                np.testing.assert_allclose(float((sd[n].double() ** 2).sum()), ref[i, 1], rtol=1e-6, err_msg=n)
    Pg, Pf, Pv = _params(sg), _params(sf), _params(sv)
    vae_stats = V.bn_stats(sg)
    data = inputs.step_batch(2, 128, 128)
    vs = OL.synthetic_vgg19_state()
    state = None
    for k in range(2):
        t = f"step{k + 1}_"
        ld, Pg, Pf, Pv, state, grads = OS.gan_step(Pg, Pf, Pv, vs, data, {}, {}, frame_spec=FRAME, video_spec=VIDEO,
                                                   vae={"eps": inputs.vae_eps(2, 78 + k), "stats": vae_stats},
                                                   uv_grad=k > 0, state=state, adam="torch2")
        vae_stats = state["stats"][2]
        assert list(ld.keys()) == [str(n) for n in f[t + "loss_names"]]
        np.testing.assert_allclose(list(ld.values()), f[t + "loss_values"], rtol=1e-4)
        for tag in ("g", "f", "v"):
            names = f[t + tag + "_grad_names"]
            assert sorted(grads[tag]) == [str(n) for n in names], tag  # u / v gradients from step 2 only
            _check_sumsq(grads[tag], names, f[t + tag + "_grad_stats"], (1e-3, 2e-2), t + tag,
                         zero=_bn_biases(sg) if tag == "g" else ())
        post = {"g": dict(Pg, **{n + ".running_mean": m for n, (m, _) in vae_stats.items()},
                          **{n + ".running_var": v for n, (_, v) in vae_stats.items()}), "f": Pf, "v": Pv}
        for tag in ("g", "f", "v"):
            names = [n for n in f[t + tag + "_post_names"] if "num_batches" not in str(n)]
            idx = [list(f[t + tag + "_post_names"]).index(n) for n in names]
            if tag == "g":  # Adamax moves the noise-gradient biases by +-lr at random, which
                # the following BatchNorm's batch mean (so its running mean, from step 2) carries
                skip = set(_bn_biases(sg))
                if k > 0:
                    skip |= {f"{b.rsplit('.', 2)[0]}.{int(b.rsplit('.', 2)[1]) + 1}.running_mean" for b in skip}
                keep = [j for j, n in enumerate(names) if str(n) not in skip]
                names, idx = [names[j] for j in keep], [idx[j] for j in keep]
            # step 2: Adamax's second update still amplifies the sign of near-zero gradient
            # elements (one BatchNorm beta, 32 elements, measured 2.5e-3); the median stays ~1e-8
            _check_sumsq(post[tag], np.array(names), f[t + tag + "_post"][idx], (1e-5, 1e-4 if k == 0 else 5e-3),
                         t + tag + " post")


# ---- G14d: the same two steps in float64, compared per tensor ----
# Per-tensor bar: relative L2 over 64 seeded elements (inputs.sample_idx) of every gradient and
# every post-step tensor <= 1e-6 (measured worst 9.7e-8 gradients, 2.8e-7 post-step; loss values
# 1.8e-8), loss values 1e-7.  In fp32 the same comparison is bounded by rounding that the VAE
# decoder amplifies ~100x by step 2 (the fp32 fixture's checks above); in float64 only the
# algorithm is left.  Exclusions, each listed (tests/golden/make_golden.py g14d):
# * the 17 conv biases right before a train-mode BatchNorm (_bn_biases): true gradient exactly 0,
#   so both sides hold rounding noise, which Adamax's sign-like first step turns into +-lr moves
#   of their post-step values;
# * from step 2 on, the running means of those BatchNorms (they average the biases' +-lr moves);
# * and no tensor, but step 1's near-zero gradient elements are set to the reference's values
#   before the optimizers (below): without that the same check gives 2.1e-6 / 6.4e-6 at step 2.
#   Adamax's first step moves an element by lr * g / (|g| + 1e-8), so for |g| ~ 1e-8 the move
#   follows the element's rounding-level value, not only its sign (measured: 9,132 listed
#   generator elements, none of them with the other sign, and the bar still needs them); the
#   override's size and reach are asserted below.
G14D_BAR = 1e-6


def _rel_samples(t, ref):
    v = t.detach().double().reshape(-1)
    got = v[inputs.sample_idx(v.numel(), 64)].numpy()
    return float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-300))


def test_gan_vae_sn_two_steps_match_reference_float64_per_tensor(monkeypatch):
    monkeypatch.setattr(OD, "SN_PER_CALL", False)  # (as above: this container's torch semantics)
    f = np.load(os.path.join(G, "gan_vae64.npz"))
    sg, sf, sv = (({k: v.double() for k, v in sd.items()}) for sd in reference_init())
    dt0 = torch.get_default_dtype()
    # the draws the float64 generator made after widening the model (the VGG stand-in, the batch,
    # the reparameterisation noise) were float64 draws
    torch.set_default_dtype(torch.float64)
    try:
        vs = OL.synthetic_vgg19_state()
        data = inputs.step_batch(2, 128, 128)
        eps = [inputs.vae_eps(2, 78 + k) for k in range(2)]
    finally:
        torch.set_default_dtype(dt0)
    Pg, Pf, Pv = _params(sg), _params(sf), _params(sv)
    vae_stats = V.bn_stats(sg)
    bn = _bn_biases(sg)
    # step 1's near-zero gradient elements (0 < |g| <= 1e-5 max|g| of their tensor) take the
    # reference's own values before the optimizers: both first steps move every element by +-lr
    # whatever |g| is, and at fp64 rounding 10 of the generator's 12.7 M elements (|g| ~ 1e-10 of
    # a 5e-4 maximum) come out with the other sign -- each then 2e-3 apart, which moved step 2's
    # losses by up to 5e-6
    override = {}
    for tag in ("g", "f", "v"):
        names = [str(n) for n in f[f"step1_{tag}_grad_names"]]
        rows = f[f"step1_{tag}_grad_small"]
        ov = {}
        for i in sorted({int(r) for r in rows[:, 0]}):
            sel = rows[rows[:, 0] == i]
            ov[names[i]] = (torch.from_numpy(sel[:, 1].astype(np.int64)), torch.from_numpy(sel[:, 2]))
        override[tag] = ov
    state, worst = None, {}
    for k in range(2):
        t = f"step{k + 1}_"
        ld, Pg, Pf, Pv, state, grads = OS.gan_step(Pg, Pf, Pv, vs, data, {}, {}, frame_spec=FRAME, video_spec=VIDEO,
                                                   vae={"eps": eps[k], "stats": vae_stats}, uv_grad=k > 0,
                                                   state=state, adam="torch2", dtype=torch.float64,
                                                   grad_override=override if k == 0 else None)
        vae_stats = state["stats"][2]
        if k == 0:
            # the override is recorded and bounded: it touches only elements that are near zero
            # in this run's OWN gradient (<= 2e-5 of the tensor's max, against the fixture's
            # 1e-5 selection), at most 1 % of any tensor (measured worst 0.27 %), and changes the sign of at most a
            # few; the step-1 gradients compared below are this run's own (before the override)
            ost = state.pop("override_stats")
            tot = {t: (sum(v[0] for v in d.values()), sum(v[1] for v in d.values())) for t, d in ost.items()}
            print(f"G14d step-1 override (listed, sign changed) per model: {tot}")
            for tag, d in ost.items():
                Pd = {"g": Pg, "f": Pf, "v": Pv}[tag]
                for name, (n_l, n_flip, rel) in d.items():
                    assert rel <= 2e-5, (tag, name, rel)
                    assert n_l <= max(16, 1e-2 * Pd[name].numel()), (tag, name, n_l)
            assert sum(t[1] for t in tot.values()) <= 32, tot
        loss_err = np.abs(np.array(list(ld.values())) - f[t + "loss_values"]) / np.abs(f[t + "loss_values"])
        worst[t + "loss"] = (float(loss_err.max()), str(f[t + "loss_names"][int(loss_err.argmax())]), float(np.median(loss_err)))
        skip = set(bn) | ({f"{b.rsplit('.', 2)[0]}.{int(b.rsplit('.', 2)[1]) + 1}.running_mean" for b in bn}
                          if k > 0 else set())
        post = {"g": dict(Pg, **{n + ".running_mean": m for n, (m, _) in vae_stats.items()},
                          **{n + ".running_var": v for n, (_, v) in vae_stats.items()}), "f": Pf, "v": Pv}
        for tag in ("g", "f", "v"):
            for kind, src in (("grad", grads[tag]), ("post", post[tag])):
                names = [str(n) for n in f[t + tag + f"_{kind}_names"]]
                S = f[t + tag + f"_{kind}_samples"]
                errs = {n: _rel_samples(src[n], S[i]) for i, n in enumerate(names)
                        if n not in skip and "num_batches" not in n}
                w = max(errs, key=errs.get)
                worst[t + tag + "_" + kind] = (errs[w], w, float(np.median(list(errs.values()))))
    for key, (e, n, med) in worst.items():
        print(f"G14d {key}: worst {e:.2e} ({n}), median {med:.2e}")
    for key, (e, n, med) in worst.items():
        assert e <= (1e-7 if key.endswith("loss") else G14D_BAR), (key, n, e)
