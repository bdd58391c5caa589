"""The SepUNet oracle (oracle/unet.py) reproduces the reference SepUNet (tests/golden/
sepunet.npz, G7): seeded init, train-mode outputs, input / parameter gradients, running
statistics.  CPU only."""
import os

import numpy as np
import torch

import inputs
from oracle import unet as OU

G = os.path.join(os.path.dirname(__file__), "golden")


def test_sepunet_oracle_matches_reference():
    f = np.load(os.path.join(G, "sepunet.npz"))
    P = OU.init_params(5)
    st = OU.fresh_stats(P)
    inp, mask, g_rgb, g_seg = inputs.sepunet_inputs()
    inp = inp.clone().requires_grad_(True)
    params = {k: v.clone().requires_grad_(True) for k, v in P.items() if "running" not in k}
    rgb, seg = OU.forward(params, st, inp, mask)
    ((rgb * g_rgb).sum() + (seg * g_seg).sum()).backward()
    np.testing.assert_allclose(rgb.detach().numpy(), f["rgb"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(seg.detach().numpy(), f["seg"], rtol=0, atol=1e-5)
    gi = inp.grad.double().reshape(-1)
    ref = f["gin"]
    np.testing.assert_allclose([float(gi.abs().sum()), float(gi.norm())], ref[1:3], rtol=1e-4)
    np.testing.assert_allclose(gi[inputs.sample_idx(gi.numel())].numpy(), ref[3:], rtol=0,
                               atol=1e-4 * float(np.abs(ref[3:]).max()))
    names = [str(n) for n in f["param_names"]]
    assert sorted(params) == names
    g2 = np.array([float((params[n].grad.double() ** 2).sum()) for n in names])
    ref2 = f["grad_stats"][:, 1]
    ok = np.abs(g2 - ref2) <= 1e-3 * ref2 + 1e-12  # (BN-preceding conv biases: ~0 both)
    assert ok.all(), [n for n, o in zip(names, ok) if not o]
    bufs = []
    for k in [str(b) for b in f["buf_names"]]:
        base, which = k.rsplit(".", 1)
        bufs.append(st[base][0 if which == "running_mean" else 1].numpy().reshape(-1))
    np.testing.assert_allclose(np.concatenate(bufs), f["bufs"], rtol=1e-4, atol=1e-6)
