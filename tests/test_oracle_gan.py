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
