"""GPU: the fused head backward (dvie_head3_bwd, csrc/head_bwd.hip) -- the backward of HRNet's
narrow-output 3x3 heads rgb_layer[2] / seg_layer[2] (reference nets/HRNet.py:410-442, 584-588)
with the hidden map's LeakyReLU derivative, data and weight gradient in one pass over the map.

* op level, through the C ABI: against torch's fp32 conv2d input / weight gradients of the same
  bf16 operands (ragged tiles: H, W not multiples of the 4 x 64 tile; a strided hidden map as in
  the stacked 896-channel buffer; cout 3 -> 8 and 20 -> 24 padded; several slabs);
* plan level: an HRNet bf16 forward + backward with the fused path against the unfused one
  (DVIE_HEAD3_FUSED=0: halo data-gradient conv + halo weight gradient) on the same weights."""
import ctypes
import os
import types

import pytest
import torch
import torch.nn.functional as F

import inputs

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(1e-30, float(b.norm())))


def _pack_wd(w, co_p, kpad):
    """data-gradient weights [c][kpad]: wd[ci][t * co_p + o] = w[o][ci][2 - i][2 - j], t = 3 i + j"""
    cout, c = w.shape[:2]
    wd = torch.zeros((c, kpad), dtype=torch.float32)
    for t in range(9):
        i, j = divmod(t, 3)
        wd[:, t * co_p:t * co_p + cout] = w[:, :, 2 - i, 2 - j].t()
    return wd


@pytest.mark.parametrize("cout,co_p", [(3, 8), (20, 24)])
@pytest.mark.parametrize("n,H,W,c,splits", [(2, 10, 100, 128, 3), (1, 8, 64, 448, 36)])
def test_head3_bwd_matches_torch(dev, cout, co_p, n, H, W, c, splits):
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    g0 = torch.Generator().manual_seed(7 + c + cout)
    hld = 2 * c  # the stacked hidden buffer: this head reads one half
    hbuf = torch.randn((n, H, W, hld), generator=g0)
    h = hbuf[..., c:2 * c].clone()  # second half
    gout = torch.zeros((n, H, W, co_p))
    gout[..., :cout] = torch.randn((n, H, W, cout), generator=g0)
    w = torch.randn((cout, c, 3, 3), generator=g0) * 0.05
    kpad = (9 * co_p + 63) // 64 * 64
    wd = _pack_wd(w, co_p, kpad)
    hb, gb, wdb = hbuf.to(torch.bfloat16).to(dev), gout.to(torch.bfloat16).to(dev), wd.to(torch.bfloat16).to(dev)
    dh = torch.full((n, H, W, hld), float("nan"), dtype=torch.bfloat16, device=dev)
    ws = torch.full((splits * co_p * 9 * c,), float("nan"), dtype=torch.float32, device=dev)
    d = L.Head3BwdDesc()
    d.g, d.h, d.wd, d.dh, d.ws = gb.data_ptr(), hb.data_ptr() + 2 * c, wdb.data_ptr(), dh.data_ptr() + 2 * c, ws.data_ptr()
    d.g_ld, d.h_ld, d.dh_ld = co_p, hld, hld
    d.n, d.hgt, d.wid, d.c = n, H, W, c
    d.cout, d.kpad, d.dy0, d.dx0 = co_p, kpad, -1, -1
    d.splits, d.dact, d.alpha = splits, L.ACT_LRELU, 0.2
    L.check(lib.dvie_head3_bwd(ctypes.byref(d), L.stream_ptr(dev)), "head3_bwd")
    torch.cuda.synchronize()
    # reference: fp32 gradients of the same (bf16-rounded) operands
    hf = hb[..., c:].float().cpu().permute(0, 3, 1, 2)
    gf = gb[..., :cout].float().cpu().permute(0, 3, 1, 2)
    wf = wdb.float().cpu()  # the bf16 weights the kernel sees, back to OIHW
    wr = torch.zeros_like(w)
    for t in range(9):
        i, j = divmod(t, 3)
        wr[:, :, 2 - i, 2 - j] = wf[:, t * co_p:t * co_p + cout].t()
    dx = torch.nn.grad.conv2d_input((n, c, H, W), wr, gf, padding=1)
    dx = dx * torch.where(hf > 0, 1.0, 0.2)
    dw = torch.nn.grad.conv2d_weight(hf, w.shape, gf, padding=1)
    got_dh = dh[..., c:].float().cpu().permute(0, 3, 1, 2)
    assert torch.isfinite(got_dh).all()
    assert torch.isnan(dh[..., :c].float()).all()  # the other half untouched
    e = rel_l2(got_dh, dx)
    assert e < 4e-3, e  # bf16 output rounding
    part = ws.view(splits, co_p, 9, c).sum(0)[:cout]  # [o][forward tap][ci]
    got_dw = part.permute(0, 2, 1).reshape(cout, c, 3, 3).cpu()
    e = rel_l2(got_dw, dw)
    assert e < 1e-5, e  # fp32 sums of the same products


def test_hrnet_head3_fused_matches_unfused(dev, monkeypatch):
    """HRNet bf16 at 64x128 (batch 2): the fused head backward against the unfused one,
    same weights and inputs.  Head 3x3 weight / bias gradients: fp32 sums of the same bf16
    products in another order (1e-4 relative L2); every other gradient (they come back through
    the bf16 hidden-map gradient, which may differ by an ulp): 2e-2; outputs identical."""
    from deep_video_interpolation_extrapolation_amd import nets
    x, seg = inputs.hrnet_input(2, 64, 128)
    gr = torch.Generator().manual_seed(3)
    w1, w2 = torch.randn((2, 3, 64, 128), generator=gr), torch.randn((2, 20, 64, 128), generator=gr)
    res = {}
    for mode in ("2", "1", "0"):  # both heads fused / the rgb head only (default) / none
        monkeypatch.setenv("DVIE_HEAD3_FUSED", mode)
        monkeypatch.setenv("DVIE_PRECISION", "bf16")
        torch.manual_seed(1024)
        m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet",
                                                precision="bf16")).to(dev)
        rgb, s = m(x.to(dev), seg.to(dev))
        ((rgb * w1.to(dev)).sum() + (s * w2.to(dev)).sum()).backward()
        torch.cuda.synchronize()
        kinds = [m.coarse_model.last_plan.bwd_arr[i].kind for i in range(m.coarse_model.last_plan.n_bwd)]
        res[mode] = (rgb.detach().float().cpu(), s.detach().float().cpu(),
                     {k: p.grad.detach().clone().cpu() for k, p in m.coarse_model.named_parameters()}, kinds)
    from deep_video_interpolation_extrapolation_amd import _lib as L
    assert [res[m][3].count(L.OP_HEAD3_BWD) for m in ("2", "1", "0")] == [2, 1, 0]
    assert torch.equal(res["2"][0], res["0"][0]) and torch.equal(res["2"][1], res["0"][1])
    ga, gb = res["2"][2], res["0"][2]
    worst = {}
    for k in gb:
        e = rel_l2(ga[k], gb[k])
        worst[k] = e
        bar = 1e-4 if k.startswith(("rgb_layer.2", "seg_layer.2")) else 2e-2
        assert e <= bar, (k, e)
    print("fused vs unfused head backward: worst relative L2", max(worst.values()), max(worst, key=worst.get))


def test_segenc_fused_forward(dev, monkeypatch):
    """The fused segmentation-encoder forward (dvie_segenc_fwd, csrc/segenc.hip; reference
    nets/HRNet.py:358-364, 533-537) inside the HRNet bf16 plan at 36x100 (ragged 4 x 64
    tiles): e1 / e2 / the encoder output in the stem buffer against torch fp32 convs of the same
    bf16 operands (4e-3 relative L2: bf16 output rounding), and the whole forward + backward
    against the unfused plan (DVIE_SEGENC_FUSED=0): outputs and gradients within 2e-2; the fused
    backward (dvie_segenc_bwd: the encoder's weight / bias gradients with d_e2, d_e1 on chip)
    against torch fp32 gradients from the plan's stored maps within 1e-2."""
    from deep_video_interpolation_extrapolation_amd import nets
    from deep_video_interpolation_extrapolation_amd import _lib as L
    x, seg = inputs.hrnet_input(2, 36, 100)
    gr = torch.Generator().manual_seed(5)
    w1, w2 = torch.randn((2, 3, 36, 100), generator=gr), torch.randn((2, 20, 36, 100), generator=gr)
    res = {}
    monkeypatch.setenv("DVIE_SEGENC_FWD", "1")  # the fused forward (the default)
    for mode in ("1", "0"):
        monkeypatch.setenv("DVIE_SEGENC_FUSED", mode)
        monkeypatch.setenv("DVIE_PRECISION", "bf16")
        torch.manual_seed(1024)
        m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet",
                                                precision="bf16")).to(dev)
        rgb, s = m(x.to(dev), seg.to(dev))
        plan = m.coarse_model.last_plan
        bufs = {b.name: b.t.detach().float().cpu().clone() for b in plan.g.buffers
                if b.t is not None and b.name.startswith(("seg0", "seg1", "feat"))}
        ((rgb * w1.to(dev)).sum() + (s * w2.to(dev)).sum()).backward()
        torch.cuda.synchronize()
        bufs["feat_grad"] = next(b for b in plan.g.buffers if b.name == "feat").g.detach().float().cpu().clone()
        kinds = [plan.fwd_arr[i].kind for i in range(len(plan.fwd_arr))]
        res[mode] = (rgb.detach().float().cpu(), s.detach().float().cpu(), bufs,
                     {k: p.grad.detach().clone().cpu() for k, p in m.coarse_model.named_parameters()}, kinds, m)
    assert res["1"][4].count(L.OP_SEGENC_FWD) == 2 and res["0"][4].count(L.OP_SEGENC_FWD) == 0
    enc = res["1"][5].coarse_model.seg_encoder
    bufs = res["1"][2]
    for k in range(2):
        t = bufs[f"seg{k}_in"].permute(0, 3, 1, 2)[:, :20]
        ref = t
        for i, (conv, act) in enumerate(((enc[0], True), (enc[2], True), (enc[4], False))):
            wq = conv.weight.detach().cpu().to(torch.bfloat16).float()
            ref = F.conv2d(ref, wq, conv.bias.detach().cpu(), padding=1)
            if act:
                ref = F.elu(ref)
            got = (bufs[f"seg{k}_e{i + 1}"] if i < 2 else bufs["feat"][..., 8 * k:8 * k + 4]).permute(0, 3, 1, 2)
            e = rel_l2(got, ref)
            assert e < 4e-3, (k, i, e)
            ref = got  # the next conv reads the stored bf16 map
    for a, b in zip(res["1"][:2], res["0"][:2]):
        assert rel_l2(a, b) < 2e-2
    ga, gb = res["1"][3], res["0"][3]
    for k in gb:
        assert rel_l2(ga[k], gb[k]) < 2e-2, (k, rel_l2(ga[k], gb[k]))
    # the fused backward (dvie_segenc_bwd) against torch fp32 on the plan's own bf16 maps:
    # dout = the stem-buffer gradient slice, e1 / e2 / the encoder input as stored
    assert res["1"][4].count(L.OP_SEGENC_BWD) == 0  # (forward list)
    ref = {k: 0.0 for k in ga if k.startswith("seg_encoder")}
    ws = [enc[i].weight.detach().cpu().to(torch.bfloat16).float() for i in (0, 2, 4)]
    for k in range(2):
        nchw = lambda t: t.permute(0, 3, 1, 2)  # noqa: E731
        xin = nchw(bufs[f"seg{k}_in"])[:, :20]
        e1, e2 = nchw(bufs[f"seg{k}_e1"]), nchw(bufs[f"seg{k}_e2"])
        dout = nchw(bufs["feat_grad"][..., 8 * k:8 * k + 4])
        d2 = torch.nn.grad.conv2d_input(e2.shape, ws[2], dout, padding=1) * torch.where(e2 > 0, 1.0, e2 + 1.0)
        d1 = torch.nn.grad.conv2d_input(e1.shape, ws[1], d2, padding=1) * torch.where(e1 > 0, 1.0, e1 + 1.0)
        for i, (gy, xx) in zip((0, 2, 4), ((d1, xin), (d2, e1), (dout, e2))):
            ref[f"seg_encoder.{i}.weight"] = ref[f"seg_encoder.{i}.weight"] + torch.nn.grad.conv2d_weight(
                xx, ws[i // 2].shape, gy, padding=1)
            ref[f"seg_encoder.{i}.bias"] = ref[f"seg_encoder.{i}.bias"] + gy.sum((0, 2, 3))
    for k, r in ref.items():
        e = rel_l2(ga[k], r)
        print(f"{k}: fused backward vs torch fp32 on the same maps {e:.2e}")
        assert e < 1e-2, (k, e)  # d_e2 / d_e1 rounded to bf16 on chip
