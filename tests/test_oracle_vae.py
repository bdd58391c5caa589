"""The CPU oracle of VAEHRNet (oracle/vaehrnet.py) reproduces the reference module
(tests/golden/vaehrnet.npz, G9): seeded initial weights, train-mode outputs (BatchNorm batch
statistics), mu / logvar, parameter gradients and running statistics.  CPU only."""
import os

import numpy as np
import torch

import inputs
from oracle import vaehrnet as V

G = os.path.join(os.path.dirname(__file__), "golden")


def run_oracle(dtype=torch.float32, masks=None):
    P = V.init_params(1024)
    stats = V.bn_stats(P)
    x, seg, gt_x, gt_seg, (g_rgb, g_seg, g_mu, g_lv) = inputs.vae_inputs()
    eps = inputs.vae_eps()
    params = {k: v.clone().to(dtype).requires_grad_(True) for k, v in P.items() if "running" not in k}
    st = {k: (a.to(dtype), b.to(dtype)) for k, (a, b) in stats.items()}
    rgb, seg_out, mu, logvar = V.forward(params, x.to(dtype), seg.to(dtype), gt_x.to(dtype), gt_seg.to(dtype),
                                         eps.to(dtype), st, masks=masks)
    ((rgb * g_rgb.to(dtype)).sum() + (seg_out * g_seg.to(dtype)).sum() + (mu * g_mu.to(dtype)).sum()
     + (logvar * g_lv.to(dtype)).sum()).backward()
    return P, params, st, (rgb, seg_out, mu, logvar)


def test_vaehrnet_oracle_matches_reference():
    f = np.load(os.path.join(G, "vaehrnet.npz"))
    P, params, st, (rgb, seg_out, mu, logvar) = run_oracle()
    names = [str(n) for n in f["param_names"]]
    assert sorted(params) == names
    cs = np.array([[float(P[n].double().sum()), float((P[n].double() ** 2).sum())] for n in names])
    np.testing.assert_allclose(cs, f["param_checksums"], rtol=1e-6, atol=1e-6)  # seeded init, same order
    np.testing.assert_allclose(mu.detach().numpy(), f["mu"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(logvar.detach().numpy(), f["logvar"], rtol=1e-4, atol=1e-5)
    for k, t in (("rgb", rgb), ("seg", seg_out)):
        v = t.detach().double().reshape(-1)
        got = v[inputs.sample_idx(v.numel())].numpy()
        ref = f[k]
        assert np.abs(got - ref[3:]).max() / np.abs(ref[3:]).max() < 1e-4, k
        np.testing.assert_allclose([float(v.abs().sum()), float(v.norm())], ref[1:3], rtol=1e-4)
    g2 = np.array([float((params[n].grad.double() ** 2).sum()) for n in names])
    ref2 = f["grad_stats"][:, 1]
    ok = np.abs(g2 - ref2) <= 1e-3 * ref2 + 1e-12  # BatchNorm-preceding conv biases: ~0
    assert ok.all(), [n for n, o in zip(names, ok) if not o]
    bufs = np.concatenate([st[k[:-len(".running_mean")]][0].numpy() if k.endswith("running_mean")
                           else st[k[:-len(".running_var")]][1].numpy() for k in [str(b) for b in f["buf_names"]]])
    np.testing.assert_allclose(bufs, f["bufs"], rtol=1e-4, atol=1e-6)
