"""GPU parity: every HIP kernel family against the CPU oracle / plain fp32 PyTorch CPU.

Tolerances (written per test): fp32 parity mode — the north-star bar, 1e-3 max-abs on
network outputs (HRNet rgb/seg), tighter on single ops; bf16 mode — relative checks
(bf16 has 8 significant bits).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import inputs
from oracle import hrnet as O
from oracle import losses as OL
from oracle import warp as OW

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / max(1e-12, float(b.abs().max())))


CONV_CASES = [
    # cin, cout, k, stride, H, W, bias
    (3, 64, 3, 1, 16, 24, True),
    (64, 64, 3, 1, 32, 48, False),
    (64, 128, 3, 2, 32, 48, False),
    (128, 64, 1, 1, 16, 24, False),
    (256, 128, 3, 2, 17, 23, False),
    (448, 3, 3, 1, 16, 16, True),
    (20, 32, 3, 1, 16, 16, True),
    (32, 4, 3, 1, 16, 16, True),
    (448, 448, 1, 1, 8, 16, True),
    (64, 256, 1, 1, 20, 36, False),
    (320, 272, 1, 1, 13, 21, False),
    (16, 96, 3, 1, 20, 70, True),
    (24, 448, 3, 1, 9, 130, False),
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_conv2d_fwd_bwd(dev, case, prec, monkeypatch):
    monkeypatch.setenv("DVIE_PRECISION", prec)
    from deep_video_interpolation_extrapolation_amd.nets.conv import Conv2d
    cin, cout, k, s, H, W, bias = case
    torch.manual_seed(0)
    m = Conv2d(cin, cout, k, s, k // 2, bias=bias)
    x = torch.randn(2, cin, H, W)
    ref = torch.nn.Conv2d(cin, cout, k, s, k // 2, bias=bias)
    ref.load_state_dict(m.state_dict())
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    m = m.to(dev)
    xg = x.to(dev).requires_grad_(True)
    y = m(xg)
    y.backward(gy.to(dev))
    torch.cuda.synchronize()
    tol = 2e-5 if prec == "fp32" else 2e-2
    assert rel_err(y, yr) < tol, ("fwd", rel_err(y, yr))
    assert rel_err(xg.grad, xr.grad) < tol * 2, ("dgrad", rel_err(xg.grad, xr.grad))
    assert rel_err(m.weight.grad, ref.weight.grad) < tol * 2, ("wgrad", rel_err(m.weight.grad, ref.weight.grad))
    if bias:
        assert rel_err(m.bias.grad, ref.bias.grad) < tol * 2


def _loss_pair(dev, fn_dvie, fn_ref, a, b):
    ag = a.to(dev).requires_grad_(True)
    v = fn_dvie(ag, b.to(dev))
    v.backward()
    ar = a.clone().requires_grad_(True)
    vr = fn_ref(ar, b)
    vr.backward()
    return float(v), float(vr), ag.grad.cpu(), ar.grad


@pytest.mark.parametrize("name", ["l1", "gdl", "ssim"])
def test_pixel_losses(dev, name):
    from deep_video_interpolation_extrapolation_amd import losses as DL
    fd = {"l1": DL.l1_loss, "gdl": DL.gdl_loss, "ssim": DL.ssim_loss}[name]
    fr = {"l1": OL.l1_loss, "gdl": OL.gdl_loss, "ssim": OL.ssim_loss}[name]
    pred, gt, _ = inputs.rgbloss_inputs()["pm1"]
    v, vr, g, gr = _loss_pair(dev, fd, fr, pred, gt)
    assert abs(v - vr) <= 1e-5 * max(1, abs(vr))
    assert rel_err(g, gr) < 1e-4
    # strided (channels-last) prediction, as HRNet outputs it
    p2 = pred.permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)
    v2, _, g2, _ = _loss_pair(dev, fd, fr, p2, gt)
    assert abs(v2 - vr) <= 1e-5 * max(1, abs(vr)) and rel_err(g2, gr) < 1e-4


def test_ssim_gradient_near_degenerate(dev):
    """Prediction ~ small negative constant, target positive: the SSIM terms
    2*mu1*mu2 + C1 and 2*sigma12 + C2 cross zero at some pixels; the gradient must stay finite
    and match autograd of the reference formula (losses.py:18-48)."""
    from deep_video_interpolation_extrapolation_amd import losses as DL
    torch.manual_seed(7)
    gt = torch.rand(2, 3, 48, 64)
    pred = -0.02 + 0.003 * torch.randn(2, 3, 48, 64)
    v, vr, g, gr = _loss_pair(dev, DL.ssim_loss, OL.ssim_loss, pred, gt)
    assert torch.isfinite(g).all() and torch.isfinite(gr).all()
    assert abs(v - vr) <= 1e-5 * max(1, abs(vr))
    assert rel_err(g, gr) < 1e-3


def test_cross_entropy(dev):
    from deep_video_interpolation_extrapolation_amd import losses as DL
    logits, onehot = inputs.ce_inputs()
    v, vr, g, gr = _loss_pair(dev, DL.seg_cross_entropy, OL.seg_ce, logits, onehot)
    assert abs(v - vr) < 1e-5
    assert rel_err(g, gr) < 1e-5


def test_psnr(dev):
    from deep_video_interpolation_extrapolation_amd import losses as DL
    pred, gt = inputs.metric_inputs()
    assert abs(float(DL.PSNR()(pred.to(dev), gt.to(dev))) - float(OL.psnr(pred, gt))) < 1e-4


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_vgg_loss(dev, prec, monkeypatch):
    monkeypatch.setenv("DVIE_PRECISION", prec)
    from deep_video_interpolation_extrapolation_amd import losses as DL
    pred, gt, _ = inputs.rgbloss_inputs()["pm1"]
    vl = DL.VGGLoss().to(dev)
    st = OL.synthetic_vgg19_state()
    v, vr, g, gr = _loss_pair(dev, lambda a, b: vl(a, b, normed=False),
                              lambda a, b: OL.vgg_loss(st, a, b, normed=False), pred, gt)
    tol = 1e-4 if prec == "fp32" else 3e-2
    assert abs(v - vr) <= tol * abs(vr)
    assert rel_err(g, gr) < (1e-3 if prec == "fp32" else 1e-1)


@pytest.mark.parametrize("shape", [(2, 5, 7, 64, 64), (3, 4, 9, 24, 40), (2, 3, 5, 20, 24)])
def test_feature_l1_nhwc_bf16(dev, shape):
    """The plan's VGG feature-L1 value (dvie_loss kind L1NHWC, losses.py:157-180) on bf16 NHWC
    maps (B, H, W, ch of a C-channel buffer) against float64 torch on the same bf16 values:
    dense rows with ch % 8 == 0 take the 16-byte kernel (also as a channel region of a wider
    buffer), ch = 20 the per-element one; both within 1e-6 relative."""
    import ctypes
    from deep_video_interpolation_extrapolation_amd import _lib as L
    B, H, W, ch, C = shape
    g = torch.Generator().manual_seed(7)
    a = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).to(dev)
    b = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).to(dev)
    lib = L.load()
    d = L.LossDesc()
    d.kind, d.a, d.b, d.dtype = L.LOSS_L1NHWC, a.data_ptr(), b.data_ptr(), L.BF16
    d.a_sn, d.a_sc, d.a_sh, d.a_sw = H * W * C, 1, W * C, C
    d.b_sn, d.b_sc, d.b_sh, d.b_sw = H * W * C, 1, W * C, C
    d.bsz, d.ch, d.h, d.w, d.weight, d.out_scale = B, ch, H, W, 1.0, 1.0
    part = torch.empty(max(1, lib.dvie_loss_partial_count(ctypes.byref(d))), dtype=torch.float64, device=dev)
    out = torch.empty(1, dtype=torch.float32, device=dev)
    d.partial, d.out = part.data_ptr(), out.data_ptr()
    L.check(lib.dvie_loss(ctypes.byref(d), L.stream_ptr(dev)), "l1nhwc")
    ref = (a[..., :ch].double() - b[..., :ch].double()).abs().mean().item()
    assert abs(float(out.item()) - ref) <= 1e-6 * ref, (float(out.item()), ref)


def test_vgg_repacks_changed_weights(dev, monkeypatch):
    """The frozen VGG19 plan packs its weights once (Plan.static_weights); an in-place weight
    update (new version counter) must be repacked: the loss after scaling features.0 by 2
    equals a fresh module's with the scaled weights."""
    monkeypatch.setenv("DVIE_PRECISION", "fp32")
    from deep_video_interpolation_extrapolation_amd import losses as DL
    pred, gt, _ = inputs.rgbloss_inputs()["pm1"]
    pred, gt = pred.to(dev), gt.to(dev)
    vl = DL.VGGLoss().to(dev)
    a = float(vl(pred, gt, normed=False))
    assert float(vl(pred, gt, normed=False)) == a  # skipped pack: same weights, same value
    w = [p for n, p in vl.named_parameters() if n.endswith("features.0.weight")]
    assert len(w) == 1
    with torch.no_grad():
        w[0].mul_(2)
    b = float(vl(pred, gt, normed=False))
    ref = DL.VGGLoss().to(dev)
    w2 = [p for n, p in ref.named_parameters() if n.endswith("features.0.weight")][0]
    with torch.no_grad():
        w2.mul_(2)
    c = float(ref(pred, gt, normed=False))
    assert b != a and abs(b - c) <= 1e-6 * abs(c)


def test_warp(dev):
    from deep_video_interpolation_extrapolation_amd.utils.net_utils import FlowWrapper
    x, flow, dout = inputs.warp_inputs()
    xg, fg = x.to(dev).requires_grad_(True), flow.to(dev).requires_grad_(True)
    y = FlowWrapper()(xg, fg)
    y.backward(dout.to(dev))
    xr, fr = x.clone().requires_grad_(True), flow.clone().requires_grad_(True)
    yr = OW.flow_warp(xr, fr)
    yr.backward(dout)
    assert float((y.cpu() - yr).abs().max()) < 1e-5
    assert float((xg.grad.cpu() - xr.grad).abs().max()) < 1e-4
    assert float((fg.grad.cpu() - fr.grad).abs().max()) < 1e-3


@pytest.mark.parametrize("with_dimg", [True, False])
@pytest.mark.parametrize("shape,far_frac", [((2, 5, 40, 136), 0.05), ((1, 3, 33, 66), 0.05), ((2, 3, 70, 200), 0.0),
                                            ((1, 4, 37, 130), 0.002), ((2, 3, 36, 128), 0.05), ((1, 3, 20, 256), 0.0),
                                            ((1, 3, 9, 64), 0.2), ((1, 3, 12, 1030), 0.0), ((2, 3, 16, 1024), 0.001)])
def test_warp_multi_tile(dev, with_dimg, shape, far_frac):
    """dvie_warp_bwd through the C ABI on frames spanning many 256-pixel row segments: a
    smooth flow of a few pixels (every sample inside its corners' 3x3 pull windows) plus a
    sparse set of large displacements (far corners and their atomics; a tile holding one
    reads from global memory, a tile without from its LDS-staged region: far_frac 0 and
    0.002 keep most tiles on the LDS path); the dimg + dflow path and the dflow-only path
    (dimg = NULL, no workspace); 3-5 channels.  Rows of a multiple of 64 pixels (whole
    64-lane waves, no partial segment) are covered too; 3 channels at even widths take the
    two-pixels-per-lane forward (paired corner-row loads on smooth waves, one-pixel loads on
    waves holding a far sample), 1030 a partial 512-pixel segment.
    Tolerances: out 1e-5, dimg 1e-4, dflow 1e-3 abs."""
    import ctypes
    from deep_video_interpolation_extrapolation_amd import _lib as L
    n, c, h, w = shape
    g = torch.Generator().manual_seed(23)
    x = torch.rand((n, c, h, w), generator=g)
    yy, xx = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32), indexing="ij")
    flow = torch.stack([torch.sin(xx / 9.0 + yy / 13.0) * 6.0 / w, torch.cos(yy / 7.0 - xx / 17.0) * 5.0 / h])
    flow = flow.unsqueeze(0).repeat(n, 1, 1, 1) + (torch.rand((n, 2, h, w), generator=g) - 0.5) * 0.02
    far = torch.rand((n, 1, h, w), generator=g) < far_frac
    flow = torch.where(far, (torch.rand((n, 2, h, w), generator=g) * 2 - 1) * 0.8, flow)
    dout = torch.randn((n, c, h, w), generator=g)
    xr, fr = x.clone().requires_grad_(True), flow.clone().requires_grad_(True)
    yr = OW.flow_warp(xr, fr)
    yr.backward(dout)

    lib = L.load()
    xd, fd, gd = x.to(dev), flow.to(dev), dout.to(dev)
    # dimg is overwritten (not accumulated): start from NaN so an unwritten cell fails
    out, dx, dfl = torch.empty_like(xd), torch.full_like(xd, float("nan")), torch.empty_like(fd)
    d = L.WarpDesc()
    d.img, d.flow, d.out, d.dout, d.dimg, d.dflow = (t.data_ptr() for t in (xd, fd, out, gd, dx, dfl))
    d.n, d.c, d.h, d.w, d.align_corners = n, c, h, w, 1
    if not with_dimg:
        d.dimg = None
    ws = torch.full((max(lib.dvie_warp_ws_floats(ctypes.byref(d)), 1),), float("nan"), device=dev)
    d.ws = ws.data_ptr()
    s = L.stream_ptr(dev)
    L.check(lib.dvie_warp_fwd(ctypes.byref(d), s), "warp fwd")
    L.check(lib.dvie_warp_bwd(ctypes.byref(d), s), "warp bwd")
    torch.cuda.synchronize()
    assert float((out.cpu() - yr.detach()).abs().max()) < 1e-5
    if with_dimg:
        assert float((dx.cpu() - xr.grad).abs().max()) < 1e-4
    assert float((dfl.cpu() - fr.grad).abs().max()) < 1e-3


def _hrnet(dev, prec, monkeypatch):
    monkeypatch.setenv("DVIE_PRECISION", prec)
    import types
    from deep_video_interpolation_extrapolation_amd import nets
    torch.manual_seed(1024)
    m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet"))
    return m.to(dev)


def test_hrnet_forward_fp32_parity(dev, monkeypatch):
    """north-star bar: outputs within 1e-3 max-abs of the CPU reference on fixed seeds."""
    m = _hrnet(dev, "fp32", monkeypatch)
    P = O.init_params(1024)
    x, seg = inputs.hrnet_input(2, 32, 64)
    with torch.no_grad():
        rgb, s = m(x.to(dev), seg.to(dev))
        rr, sr = O.forward(P, torch.cat([x, seg], 1))
    assert float((rgb.cpu() - rr).abs().max()) < 1e-3
    assert float((s.cpu() - sr).abs().max()) < 1e-3


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_hrnet_frame_parts_match_concatenated(dev, monkeypatch, prec):
    """HRNet.forward_split with the frames and segmentations as per-frame tensors (the plan's
    input ops read them in place; the two-frame rgb op through the EW_NCHW src1 split) is
    bit-identical to the concatenated input, for separate tensors and for channel views of
    one tensor, and its backward gives the same parameter gradients."""
    m = _hrnet(dev, prec, monkeypatch)
    x, seg = inputs.hrnet_input(2, 32, 64)
    x, seg = x.to(dev), seg.to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    w1, w2 = torch.randn((2, 3, 32, 64), generator=g, device=dev), torch.randn((2, 20, 32, 64), generator=g, device=dev)

    def run(xi, si):
        for p in m.parameters():
            p.grad = None
        rgb, s = m(xi, si)
        ((rgb * w1).sum() + (s * w2).sum()).backward()
        return rgb.detach().clone(), s.detach().clone(), [p.grad.clone() for p in m.parameters() if p.grad is not None]

    ref = run(x, seg)
    sep = run([x[:, :3].contiguous(), x[:, 3:].contiguous()], [seg[:, :20].contiguous(), seg[:, 20:].contiguous()])
    views = run([x[:, :3], x[:, 3:]], [seg[:, :20], seg[:, 20:]])
    for got in (sep, views):
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
        assert len(got[2]) == len(ref[2]) and all(torch.equal(a, b) for a, b in zip(got[2], ref[2]))


def test_hrnet_backward_fp32_parity(dev, monkeypatch):
    """Parameter gradients vs an fp64 oracle's autograd on the same activation branches.

    An activation that fp64 puts at +1e-9 and fp32 at -1e-9 flips LeakyReLU's derivative
    (1 vs 0.2) at that pixel, which moves single gradient entries by O(1) relative
    (observed: 1 such flip in ~5e6 activations, |a| = 7.9e-9).  The fp64 oracle therefore
    takes the branches the HIP forward took (Plan.activation_signs); what remains is fp32
    rounding.  Metric: per-tensor relative L2.  Bars: every tensor <= 1e-4, median <= 1e-5."""
    m = _hrnet(dev, "fp32", monkeypatch)
    P0 = O.init_params(1024)
    x, seg = inputs.hrnet_input(2, 32, 64)
    g = torch.Generator().manual_seed(5)
    w1 = torch.randn((2, 3, 32, 64), generator=g)
    w2 = torch.randn((2, 20, 32, 64), generator=g)
    rgb, s = m(x.to(dev), seg.to(dev))
    ((rgb * w1.to(dev)).sum() + (s * w2.to(dev)).sum()).backward()
    P = {k: v.double().clone().requires_grad_(True) for k, v in P0.items()}
    masks = m.coarse_model.last_plan.activation_signs()
    rr, sr = O.forward(P, torch.cat([x, seg], 1).double(), masks=masks)
    ((rr * w1.double()).sum() + (sr * w2.double()).sum()).backward()
    named = dict(m.coarse_model.named_parameters())
    errs = {}
    for k in P0:
        a, b = named[k].grad.detach().cpu().double(), P[k].grad
        errs[k] = float((a - b).norm() / b.norm())
    worst = max(errs, key=errs.get)
    med = float(np.median(list(errs.values())))
    print(f"grad rel-L2: median {med:.2e}, worst {errs[worst]:.2e} ({worst})")
    assert errs[worst] <= 1e-4, (worst, errs[worst])
    assert med <= 1e-5, med


def test_hrnet_bf16_close_to_fp32(dev, monkeypatch):
    m = _hrnet(dev, "bf16", monkeypatch)
    P = O.init_params(1024)
    x, seg = inputs.hrnet_input(2, 32, 64)
    with torch.no_grad():
        rgb, s = m(x.to(dev), seg.to(dev))
        rr, sr = O.forward(P, torch.cat([x, seg], 1))
    assert torch.isfinite(rgb).all() and torch.isfinite(s).all()
    assert rel_err(rgb, rr) < 5e-2 and rel_err(s, sr) < 5e-2
