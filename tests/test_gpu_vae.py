"""GPU parity of VAEHRNet (reference nets/HRNet.py:702-1061): encoder / decoder plans
(ConvTranspose2d as strided data-gradient phases, train-mode BatchNorm), the Linear layers
as 1x1 convs, the HIP reparameterisation and the HRNet trunk with the decoded feature in
its stem, against the fp64 oracle (oracle/vaehrnet.py, itself pinned to the reference by
tests/golden/vaehrnet.npz) evaluated on the HIP run's LeakyReLU branches.

Tolerances: outputs and mu / logvar 1e-5 relative L2; parameter gradients 1e-4 relative L2
(3e-4 through train-mode BatchNorm; BatchNorm-preceding conv biases: zero true gradient,
compared absolutely)."""
import os
import types

import numpy as np
import pytest
import torch

import inputs
from oracle import vaehrnet as V

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(1e-30, float(b.norm())))


def make(prec, dev):
    os.environ["DVIE_PRECISION"] = prec
    from deep_video_interpolation_extrapolation_amd import nets
    torch.manual_seed(1024)
    return nets.VAEHRNet(types.SimpleNamespace(syn_type="inter", highres_large=False, precision=prec)).to(dev)


def masks_of(m):
    out = dict(m.last_plan.activation_signs())  # the HRNet trunk
    for r in (m._enc, m._dec):
        out.update(r.last_plan.activation_signs())
    return out


def test_vaehrnet_fp32_matches_oracle(dev):
    m = make("fp32", dev)
    m.train()
    x, seg, gt_x, gt_seg, (g_rgb, g_seg, g_mu, g_lv) = inputs.vae_inputs()
    eps = inputs.vae_eps()
    rgb, seg_out, mu, logvar = m.forward_vae(x.to(dev), seg.to(dev), gt_x.to(dev), gt_seg.to(dev), eps=eps.to(dev))
    ((rgb * g_rgb.to(dev)).sum() + (seg_out * g_seg.to(dev)).sum() + (mu * g_mu.to(dev)).sum()
     + (logvar * g_lv.to(dev)).sum()).backward()
    torch.cuda.synchronize()

    from test_oracle_vae import run_oracle
    P, params, st, (r_rgb, r_seg, r_mu, r_lv) = run_oracle(torch.float64, masks=masks_of(m))
    for got, ref, tag in ((mu, r_mu, "mu"), (logvar, r_lv, "logvar"), (rgb, r_rgb, "rgb"), (seg_out, r_seg, "seg")):
        e = rel_l2(got.detach(), ref.detach())
        assert e < 1e-5, (tag, e)
    named = dict(m.named_parameters())
    errs = {}
    for k, v in params.items():
        g = named[k].grad
        assert g is not None, k
        if k.endswith(".bias") and k.startswith("vae_") and f"{k.rsplit('.', 2)[0]}.{int(k.split('.')[1]) + 1}.running_mean" in P:
            assert float(g.abs().max()) < 1e-4, k  # conv bias before BatchNorm: zero gradient
            continue
        errs[k] = rel_l2(g, v.grad)
    # every LeakyReLU branch (encoder, decoder, trunk) is imposed on the fp64 oracle: only fp32
    # rounding remains.  1e-4 per tensor; 3e-4 for the encoder / decoder / FC tensors, whose
    # gradient comes back through train-mode BatchNorm backward (cancelling in fp32)
    worst = max(errs, key=errs.get)
    print(f"VAEHRNet gradients vs fp64 oracle on the same branches: relative L2 median "
          f"{np.median(list(errs.values())):.2e}, worst {errs[worst]:.2e} ({worst})")
    for k, e in errs.items():
        assert e <= (3e-4 if k.startswith(("vae_", "mu_fc", "logvar_fc")) else 1e-4), (k, e)
    sd = m.state_dict()
    for name, (rm, rv) in st.items():
        assert rel_l2(sd[name + ".running_mean"], rm) < 1e-5, name
        assert rel_l2(sd[name + ".running_var"], rv) < 1e-5, name


def test_vaehrnet_bf16_close_and_eval(dev):
    x, seg, gt_x, gt_seg, _ = inputs.vae_inputs()
    eps = inputs.vae_eps().to(dev)
    outs = []
    for prec in ("fp32", "bf16"):
        m = make(prec, dev)
        m.train()
        outs.append(m.forward_vae(x.to(dev), seg.to(dev), gt_x.to(dev), gt_seg.to(dev), eps=eps))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.isfinite(b).all()
        assert rel_l2(b.detach(), a.detach()) < 5e-2
    m.eval()  # z ~ N(0, 1), no encoder; mu = logvar = None as in the reference
    with torch.no_grad():
        rgb, seg_out, mu, lv = m(torch.cat([x, seg], 1).to(dev))
    assert mu is None and lv is None and torch.isfinite(rgb).all() and rgb.shape == (2, 3, 128, 128)
