"""The CPU oracle of the discriminators (oracle/disc.py) reproduces the reference's
FrameDiscriminator / VideoDiscriminator (tests/golden/disc.npz, G6): seeded init, train-
mode scores (BatchNorm batch statistics), input gradients, parameter gradients, running
statistics, hinge losses and eval-mode scores.  CPU only."""
import os

import numpy as np
import pytest
import torch

import inputs
from oracle import disc as OD

G = os.path.join(os.path.dirname(__file__), "golden")
CASES = [("frame", OD.FRAME, 31), ("video", OD.VIDEO, 32)]


def run_oracle(tag, spec_fn, seed, H, W):
    spec = spec_fn(23)
    P = OD.init_params(spec, seed)
    stats = {k[:-len(".running_mean")]: (P[k].clone(), P[k[:-4] + "var"].clone())
             for k in P if k.endswith("running_mean")}
    x, seg, ix, iseg, gout = inputs.disc_inputs(2, H, W)
    ins = [x, seg] + ([ix, iseg] if tag == "video" else [])
    ins = [v.clone().requires_grad_(True) for v in ins]
    params = {k: v.clone().requires_grad_(True) for k, v in P.items() if "running" not in k}
    score = OD.forward(params, spec, torch.cat(ins, 1), training=True, stats=stats)
    score.backward(gout)
    with torch.no_grad():
        ev = OD.forward(params, spec, torch.cat([v.detach() for v in ins], 1), training=False, stats=stats)
    return score, ins, params, stats, ev


@pytest.mark.parametrize("tag,spec_fn,seed", CASES)
@pytest.mark.parametrize("hw", [(128, 128), (128, 256)])
def test_disc_oracle_matches_reference(tag, spec_fn, seed, hw):
    f = np.load(os.path.join(G, "disc.npz"))
    t = f"{tag}_{hw[0]}x{hw[1]}"
    score, ins, params, stats, ev = run_oracle(tag, spec_fn, seed, *hw)
    np.testing.assert_allclose(score.detach().numpy(), f[t + "_score"], rtol=1e-4, atol=1e-5)
    for k, v in enumerate(ins):
        gv = v.grad.double().reshape(-1)
        got = np.concatenate([[float(gv.sum()), float(gv.abs().sum()), float(gv.norm())],
                              gv[inputs.sample_idx(gv.numel())].numpy()])
        ref = f[t + f"_gin{k}"]
        scale = float(np.abs(ref[3:]).max()) + 1e-30
        assert np.abs(got[3:] - ref[3:]).max() / scale < 1e-3, (k, np.abs(got[3:] - ref[3:]).max() / scale)
        np.testing.assert_allclose(got[1:3], ref[1:3], rtol=1e-3)
    names = [str(n) for n in f[t + "_param_names"]]
    assert sorted(params) == names
    g2 = np.array([float((params[n].grad.double() ** 2).sum()) for n in names])
    ref2 = f[t + "_grad_stats"][:, 1]
    # BatchNorm-preceding conv biases have exactly-zero true gradient: compare absolutely
    ok = np.abs(g2 - ref2) <= 1e-3 * ref2 + 1e-12
    assert ok.all(), [n for n, o in zip(names, ok) if not o]
    bufs = np.concatenate([torch.stack([stats[k[:-len(".running_mean")]][0]]).numpy().reshape(-1)
                           if k.endswith("running_mean") else stats[k[:-len(".running_var")]][1].numpy().reshape(-1)
                           for k in [str(b) for b in f[t + "_buf_names"]]])
    np.testing.assert_allclose(bufs, f[t + "_bufs"], rtol=1e-4, atol=1e-6)
    hinge = [float(OD.gan_scalar_loss(score.detach(), 1.5, True)), float(OD.gan_scalar_loss(score.detach(), 1.5, False))]
    np.testing.assert_allclose(hinge, f[t + "_hinge"], rtol=1e-5)
    np.testing.assert_allclose(ev.numpy(), f[t + "_score_eval"], rtol=1e-4, atol=1e-5)


G8 = [("FrameLocalDiscriminator", 51), ("FrameSNDiscriminator", 52), ("FrameSNLocalDiscriminator", 53),
      ("VideoLocalDiscriminator", 54), ("VideoSNDiscriminator", 55), ("VideoSNLocalDiscriminator", 56)]


def run_variant(cls, seed, uvgrad, dtype=torch.float32, masks=None):
    """oracle forward + backward of a G8 variant at 128x128 (seg_disc); `uvgrad`: SpectralNorm
    u / v require grad (the state after InterGANNet's set_net_grad(True))"""
    spec = OD.SPECS[cls](23)
    P = OD.init_params(spec, seed)
    stats = {k[:-len(".running_mean")]: (P[k].clone().to(dtype), P[k[:-4] + "var"].clone().to(dtype))
             for k in P if k.endswith("running_mean")}
    x, seg, ix, iseg, gout = inputs.disc_inputs(2, 128, 128)
    ins = [x, seg] + ([ix, iseg] if cls.startswith("Video") else [])
    ins = [v.clone().to(dtype).requires_grad_(True) for v in ins]
    params = {k: v.clone().to(dtype).requires_grad_(uvgrad or not k.endswith(("weight_u", "weight_v")))
              for k, v in P.items() if "running" not in k}
    out = OD.forward(params, spec, torch.cat(ins, 1), training=True, stats=stats, masks=masks)
    if out.dim() > 1:
        gout = inputs.disc_map_grad(tuple(out.shape))
    out.backward(gout.to(dtype))
    return out, ins, params, stats, P, gout


@pytest.mark.parametrize("cls,seed", G8)
@pytest.mark.parametrize("uvgrad", [False, True])
def test_disc_variant_oracle_matches_reference(cls, seed, uvgrad):
    """local (map output) and SpectralNorm discriminators vs tests/golden/disc_sn.npz (G8):
    output, input gradients, parameter gradients (u / v ones too once trainable), u / v after
    the forward's power iteration, BatchNorm running statistics."""
    if uvgrad and "SN" not in cls:
        pytest.skip("no SpectralNorm")
    f = np.load(os.path.join(G, "disc_sn.npz"))
    t = cls + ("_uvgrad" if uvgrad else "")
    out, ins, params, stats, _, _ = run_variant(cls, seed, uvgrad)
    np.testing.assert_allclose(out.detach().numpy(), f[t + "_score"], rtol=1e-4, atol=1e-5)
    for k, v in enumerate(ins):
        gv = v.grad.double().reshape(-1)
        got = gv[inputs.sample_idx(gv.numel())].numpy()
        ref = f[t + f"_gin{k}"]
        assert np.abs(got - ref[3:]).max() / (np.abs(ref[3:]).max() + 1e-30) < 1e-3, k
        np.testing.assert_allclose([float(gv.abs().sum()), float(gv.norm())], ref[1:3], rtol=1e-3)
    names = [str(n) for n in f[t + "_param_names"]]
    assert sorted(n for n, p in params.items() if p.grad is not None) == names
    g2 = np.array([float((params[n].grad.double() ** 2).sum()) for n in names])
    ref2 = f[t + "_grad_stats"][:, 1]
    ok = np.abs(g2 - ref2) <= 1e-3 * ref2 + 1e-12  # BatchNorm-preceding conv biases: ~0
    assert ok.all(), [n for n, o in zip(names, ok) if not o]
    if t + "_uv_names" in f.files:
        uv = np.concatenate([params[str(k)].detach().numpy().reshape(-1) for k in f[t + "_uv_names"]])
        np.testing.assert_allclose(uv, f[t + "_uv"], rtol=1e-4, atol=1e-6)
    if t + "_buf_names" in f.files:
        bufs = np.concatenate([stats[k[:-len(".running_mean")]][0].numpy() if k.endswith("running_mean")
                               else stats[k[:-len(".running_var")]][1].numpy()
                               for k in [str(b) for b in f[t + "_buf_names"]]])
        np.testing.assert_allclose(bufs, f[t + "_bufs"], rtol=1e-4, atol=1e-6)


def test_adam_101_matches_torch_adam_at_zero_eps():
    """The 1.0.1 Adam form and torch 2.x Adam differ only in where eps enters
    (sqrt(v) + eps vs sqrt(v)/sqrt(bc2) + eps): with eps = 0 they must agree."""
    g = torch.Generator().manual_seed(3)
    w0 = torch.randn(50, generator=g)
    p, st = {"w": w0.clone()}, None
    ref = torch.nn.Parameter(w0.clone())
    opt = torch.optim.Adam([ref], lr=1e-3, eps=0.0)
    for it in range(3):
        grad = torch.randn(50, generator=g)
        p, st = OD.adam_101(p, {"w": grad}, 1e-3, st, eps=0.0)
        ref.grad = grad.clone()
        opt.step()
    assert float((p["w"] - ref.detach()).abs().max()) < 1e-6
