"""The CPU oracle reproduces the reference's own outputs (golden fixtures made by
tests/golden/make_golden.py from /root/reference)."""
import os

import numpy as np
import pytest
import torch

import inputs
from oracle import hrnet, losses, step, warp

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name))


def test_hrnet_init_matches_reference():
    f = load("hrnet_fwd.npz")
    sd = hrnet.init_params(1024)
    assert int(f["n_params"]) == sum(v.numel() for v in sd.values()) == 9936155
    names = [str(n) for n in f["param_names"]]
    assert sorted(sd) == names
    cs = np.array([[float(sd[n].double().sum()), float((sd[n].double() ** 2).sum())] for n in names])
    np.testing.assert_allclose(cs, f["param_checksums"], rtol=1e-12, atol=1e-12)


def test_hrnet_forward_matches_reference():
    f = load("hrnet_fwd.npz")
    P = hrnet.init_params(1024)
    x, seg = inputs.hrnet_input(2, 16, 32)
    with torch.no_grad():
        rgb, s = hrnet.forward(P, torch.cat([x, seg], 1))
    np.testing.assert_allclose(rgb.numpy(), f["rgb"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(s.numpy(), f["seg"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("tag", ["pm1", "z1", "normed"])
def test_rgbloss_matches_reference(tag):
    f = load("rgbloss.npz")
    vs = losses.synthetic_vgg19_state()
    pred, gt, normed = inputs.rgbloss_inputs()[tag]
    pred = pred.clone().requires_grad_(True)
    d = losses.rgb_loss(vs, pred, gt, normed)
    for k, v in d.items():
        key = k.replace("coarse_", "")
        (g,) = torch.autograd.grad(v, pred, retain_graph=True)
        assert abs(v.item() - float(f[f"{tag}_{key}"])) <= 1e-5 * max(1.0, abs(float(f[f"{tag}_{key}"])))
        np.testing.assert_allclose(g.numpy(), f[f"{tag}_{key}_grad"], rtol=1e-4, atol=1e-7)


def test_ce_matches_reference():
    f = load("rgbloss.npz")
    logits, onehot = inputs.ce_inputs()
    logits = logits.clone().requires_grad_(True)
    ce = losses.seg_ce(logits, onehot)
    (g,) = torch.autograd.grad(ce, logits)
    assert abs(ce.item() - float(f["ce"])) < 1e-6
    np.testing.assert_allclose(g.numpy(), f["ce_grad"], atol=1e-8)


def test_warp_matches_reference():
    f = load("warp.npz")
    x, flow, dout = inputs.warp_inputs()
    x = x.clone().requires_grad_(True)
    flow = flow.clone().requires_grad_(True)
    y = warp.flow_warp(x, flow)
    gx, gf = torch.autograd.grad(y, (x, flow), dout)
    np.testing.assert_allclose(y.detach().numpy(), f["out"], atol=1e-6)
    np.testing.assert_allclose(gx.numpy(), f["dx"], atol=1e-5)
    np.testing.assert_allclose(gf.numpy(), f["dflow"], atol=1e-4)


def test_metrics_match_reference():
    f = load("metrics.npz")
    pred, gt = inputs.metric_inputs()
    assert abs(losses.psnr(pred, gt).item() - float(f["psnr"])) < 1e-4
    assert abs(losses.ssim_loss(pred, gt).item() - float(f["ssim"])) < 1e-6
    a, b = inputs.iou_inputs()
    assert abs(((a == b).float().sum() / a.numel()).item() - float(f["iou"])) < 1e-7
    vs = losses.synthetic_vgg19_state()
    assert abs(losses.vgg_cosine(vs, pred * 2 - 1, gt * 2 - 1, normed=False).item() - float(f["vgg_cos"])) < 1e-5


def test_inter_step_matches_reference():
    f = load("step.npz")
    P = hrnet.init_params(1024)
    data = inputs.step_batch(2, 32, 64)
    ld, grads, new, _, (rgb, seg) = step.inter_step(P, losses.synthetic_vgg19_state(), data)
    names = [str(n) for n in f["loss_names"]]
    assert names == list(ld.keys())
    np.testing.assert_allclose(np.array(list(ld.values())), f["loss_values"], rtol=2e-5)
    pn = [str(n) for n in f["param_names"]]
    gs = np.array([[float(grads[n].double().sum()), float((grads[n].double() ** 2).sum()), float(grads[n].abs().max())]
                   for n in pn])
    np.testing.assert_allclose(gs[:, 1], f["grad_stats"][:, 1], rtol=1e-3)
    np.testing.assert_allclose(gs[:, 2], f["grad_stats"][:, 2], rtol=1e-3, atol=1e-9)
    post = np.array([[float(new[n].double().sum()), float((new[n].double() ** 2).sum())] for n in pn])
    np.testing.assert_allclose(post, f["post_checksums"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(rgb.numpy()[:, :, ::4, ::4], f["rgb"], atol=1e-5)
