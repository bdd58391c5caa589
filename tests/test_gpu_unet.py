"""GPU parity of the UNet family (reference nets/UNet.py, nets/SepUNet.py) and of the
bilinear upsample kernel in both align_corners modes.

SepUNet fp32 plan vs the fp64 oracle (oracle/unet.py, pinned to the reference by
tests/golden/sepunet.npz) evaluated on the HIP forward's LeakyReLU branches (see
test_gpu_gan for why); bf16 close to fp32; UNet raises the reference's channel mismatch.
"""
import os
import types

import pytest
import torch
import torch.nn.functional as F

import inputs
from oracle import unet as OU

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(1e-30, float(b.norm())))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("shape", [((5, 7), (10, 14)), ((3, 4), (17, 9)), ((8, 16), (16, 32))])
def test_bilinear_upsample_and_adjoint(dev, align, shape, dtype):
    from deep_video_interpolation_extrapolation_amd import engine as E
    (h, w), (H, W) = shape
    g = E.Graph(dtype)
    a = g.buffer("a", h, w, 8)
    g.input_nchw(E.R(a), "x", ext_c=8, requires_grad=True)
    u = g.buffer("u", H, W, 8)
    g.fuse([E.R(a)], E.R(u), align=align)
    g.output_nchw("y", E.R(u), 8)
    plan = g.compile(2, dev, backward=True)
    gen = torch.Generator().manual_seed(9)
    x = torch.randn((2, 8, h, w), generator=gen)
    gy = torch.randn((2, 8, H, W), generator=gen)
    xr = x.clone().requires_grad_(True)
    yr = F.interpolate(xr, size=(H, W), mode="bilinear", align_corners=align)
    yr.backward(gy)
    xd = x.to(dev)
    y = torch.empty((2, 8, H, W), device=dev)
    gx = torch.empty((2, 8, h, w), device=dev)
    plan.set_input("x", xd)
    plan.set_output_nchw("y", y)
    plan.run_forward()
    plan.set_output_grad("y", gy.to(dev))
    plan.set_input_grad("x", gx)
    plan.run_backward()
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 3e-2  # bf16 storage of x, y and the gradients
    assert float((y.cpu() - yr.detach()).abs().max()) < tol * 4
    assert float((gx.cpu() - xr.grad).abs().max()) < tol * 40


def make_sepunet(prec, dev, seed=5):
    os.environ["DVIE_PRECISION"] = prec
    from deep_video_interpolation_extrapolation_amd import nets
    torch.manual_seed(seed)
    return nets.SepUNet(types.SimpleNamespace(precision=prec)).to(dev)


def test_sepunet_fp32_matches_oracle(dev):
    m = make_sepunet("fp32", dev)
    P = OU.init_params(5)
    sd = m.state_dict()
    for k, v in P.items():
        assert torch.equal(sd[k].cpu(), v), k
    inp, mask, g_rgb, g_seg = inputs.sepunet_inputs()
    rgb, seg = m(inp.to(dev), fg_mask=mask.to(dev))
    ((rgb * g_rgb.to(dev)).sum() + (seg * g_seg.to(dev)).sum()).backward()
    torch.cuda.synchronize()
    masks = m.last_plan.activation_signs()
    st = OU.fresh_stats(P, torch.float64)
    params = {k: v.double().clone().requires_grad_(True) for k, v in P.items() if "running" not in k}
    rr, sr = OU.forward(params, st, inp.double(), mask.double(), masks=masks)
    ((rr * g_rgb.double()).sum() + (sr * g_seg.double()).sum()).backward()
    assert rel_l2(rgb.detach(), rr.detach()) < 1e-5, rel_l2(rgb.detach(), rr.detach())
    assert rel_l2(seg.detach(), sr.detach()) < 1e-5, rel_l2(seg.detach(), sr.detach())
    named = dict(m.named_parameters())
    bn_pre = {c for c, _, _, _, bn in OU.conv_specs() if bn}
    for k, v in params.items():
        if k.endswith(".bias") and k[:-5] in bn_pre:  # conv bias before BatchNorm: zero true gradient
            assert float(named[k].grad.abs().max()) < 1e-3 * float(named[k[:-5] + ".weight"].grad.abs().max()), k
            continue
        e = rel_l2(named[k].grad, v.grad)
        assert e < 2e-4, (k, e)
    for name, (rm, rv) in st.items():
        assert rel_l2(sd[name + ".running_mean"], rm) < 1e-4, name
        assert rel_l2(sd[name + ".running_var"], rv) < 1e-4, name
    assert int(sd["seg_encoder.sequence.1.num_batches_tracked"]) == 2  # called once per frame


def test_sepunet_bf16_close_to_fp32(dev):
    inp, mask, _, _ = inputs.sepunet_inputs()
    a = make_sepunet("fp32", dev)(inp.to(dev), fg_mask=mask.to(dev))
    b = make_sepunet("bf16", dev)(inp.to(dev), fg_mask=mask.to(dev))
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.isfinite(y).all()
        assert rel_l2(y.detach(), x.detach()) < 5e-2, rel_l2(y.detach(), x.detach())


def test_unet_raises_reference_channel_mismatch(dev):
    from deep_video_interpolation_extrapolation_amd import nets
    u = nets.UNet(types.SimpleNamespace())
    with pytest.raises(RuntimeError, match="512"):
        u(torch.zeros(1, 46, 32, 64, device=dev))
