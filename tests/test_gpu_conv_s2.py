"""GPU: the stride-2 3x3 forward convolution (csrc/conv_s2.hip, phase-split halo) through the
C ABI (dvie_conv2d_fwd) against torch's fp32 conv2d(stride=2, padding=1) on the same bf16
operands: ragged output tiles (rows not a multiple of 4, columns not of 64), odd input sizes,
channel slices of wider buffers (x_ld > c, y_ld > cout), output channels that are not a multiple
of the 64 / 128 / 256-channel tile, bias, residual and LeakyReLU.  HRNet's downsampling convs
(reference nets/HRNet.py:166-194, 444-477).  Bar: 4e-3 relative L2 (bf16 output rounding);
every byte outside the written region unchanged; the launch trace names the kernel."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(1e-30, float(b.norm())))


CASES = [  # n, ih, iw, c, x_ld, cout, y_ld, res, act
    (2, 17, 70, 16, 16, 24, 24, True, True),
    (1, 64, 130, 64, 96, 128, 136, False, True),
    (2, 33, 129, 128, 128, 256, 256, True, True),
    (1, 40, 64, 32, 32, 64, 64, False, False),
    (8, 64, 128, 64, 64, 256, 256, True, False),
]


@pytest.mark.parametrize("n,ih,iw,c,x_ld,cout,y_ld,res,act", CASES)
def test_conv_s2_matches_torch(dev, n, ih, iw, c, x_ld, cout, y_ld, res, act):
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(17 + c + cout)
    oh, ow = (ih - 1) // 2 + 1, (iw - 1) // 2 + 1
    xb = torch.randn((n, ih, iw, x_ld), generator=g).to(torch.bfloat16)
    w = (torch.randn((cout, c, 3, 3), generator=g) * (2.0 / (9 * c)) ** 0.5).to(torch.bfloat16)
    bias = torch.randn((cout,), generator=g) * 0.1
    kpad = (9 * c + 63) // 64 * 64
    wp = torch.zeros((cout, kpad), dtype=torch.bfloat16)
    wp[:, :9 * c] = w.permute(0, 2, 3, 1).reshape(cout, 9 * c)  # [co][t c + ci], t = 3 i + j
    rb = torch.randn((n, oh, ow, y_ld), generator=g).to(torch.bfloat16)
    y0 = torch.randn((n, oh, ow, y_ld), generator=g).to(torch.bfloat16)  # sentinel contents
    xd, wd, bd, rd, yd = (t.to(dev) for t in (xb, wp, bias, rb, y0.clone()))
    d = L.ConvDesc()
    d.x, d.w, d.y, d.bias = xd.data_ptr(), wd.data_ptr(), yd.data_ptr(), bd.data_ptr()
    d.res, d.z = (rd.data_ptr() if res else None), None
    d.x_ld, d.y_ld, d.res_ld, d.z_ld = x_ld, y_ld, y_ld if res else 0, 0
    d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, ih, iw, c, kpad, cout
    d.oh, d.ow, d.sy, d.sx = oh, ow, 2, 2
    d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = 3, 3, -1, -1, 1, 1
    d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = oh, ow, 1, 1, 0, 0
    d.act, d.dact, d.beta, d.dtype, d.out_f32 = (L.ACT_LRELU if act else L.ACT_NONE), 0, 0, L.BF16, 0
    d.alpha = 0.2
    lib.dvie_trace_kernels(1)
    L.check(lib.dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(L.stream_ptr(dev))), "conv s2")
    torch.cuda.synchronize()
    names = lib.dvie_traced_kernels().decode()
    lib.dvie_trace_kernels(0)
    assert "conv_s2_kernel" in names, names
    ref = F.conv2d(xb[..., :c].float().permute(0, 3, 1, 2), w.float(), bias, stride=2, padding=1)
    if res:
        ref = ref + rb[..., :cout].float().permute(0, 3, 1, 2)
    if act:
        ref = F.leaky_relu(ref, 0.2)
    got = yd.cpu()
    e = rel_l2(got[..., :cout].float().permute(0, 3, 1, 2), ref)
    print(f"conv_s2 n{n} {ih}x{iw} {c}->{cout}: rel L2 {e:.2e} ({names})")
    assert e < 4e-3, e
    assert torch.equal(got[..., cout:], y0[..., cout:])  # channels past cout untouched


# ---- the one-launch stride-2 data gradient (dvie_conv_desc.phc, csrc/conv_halo.hip PH4) ----
PH4 = ((0, 0), (1, 1), (0, 1), (1, 0))  # include/dvie.h: phase of output channel block q

DG_CASES = [  # n, H, W (the data gradient's dx size), cin, dx_ld, cout (dy channels), dy_ld, beta, dact, res
    (2, 34, 130, 64, 64, 128, 128, True, True, False),
    (1, 33, 129, 64, 96, 128, 128, False, True, False),  # odd sizes: dx rows / cols past the last phase skipped
    (2, 64, 128, 256, 256, 128, 128, True, True, False),  # transition1.1
    (1, 40, 70, 128, 128, 256, 264, False, False, True),
    (2, 32, 64, 64, 64, 256, 256, True, False, False),
    (1, 18, 66, 32, 32, 64, 64, False, True, True),
    (8, 128, 256, 64, 64, 128, 128, True, True, False),  # fuse_layers.1.0 at the bench shape / 2
]


@pytest.mark.parametrize("n,H,W,cin,dx_ld,cout,dy_ld,beta,dact,res", DG_CASES)
def test_conv_s2_dgrad_one_launch_matches_torch(dev, n, H, W, cin, dx_ld, cout, dy_ld, beta, dact, res):
    """dx = conv2d(stride 2, padding 1)'s input gradient (torch autograd, fp32) from bf16 dy and
    weights, all four output phases from ONE dvie_conv2d_fwd launch, with the epilogue
    operands the engine uses (accumulate onto dx, LeakyReLU derivative, residual); weights packed
    here from their definition (row block q = phase PH4[q], tap (i, j) = forward (a+1-2i,
    b+1-2j)), not by the engine's pack."""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(7 + cin + 3 * cout + H)
    oh, ow = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dy = torch.randn((n, oh, ow, dy_ld), generator=g).to(torch.bfloat16)
    w = (torch.randn((cout, cin, 3, 3), generator=g) * (2.0 / (9 * cin)) ** 0.5).to(torch.bfloat16)
    kpad = (4 * cout + 63) // 64 * 64
    wp = torch.zeros((4 * cin, kpad), dtype=torch.bfloat16)
    for q, (a, b) in enumerate(PH4):
        for i in range(2):
            for j in range(2):
                kh, kw = a + 1 - 2 * i, b + 1 - 2 * j
                if 0 <= kh < 3 and 0 <= kw < 3:
                    t = 2 * i + j
                    wp[q * cin:(q + 1) * cin, t * cout:(t + 1) * cout] = w[:, :, kh, kw].t()
    y0 = torch.randn((n, H, W, dx_ld), generator=g).to(torch.bfloat16)
    z = torch.randn((n, H, W, dx_ld), generator=g).to(torch.bfloat16)
    rb = torch.randn((n, H, W, dx_ld), generator=g).to(torch.bfloat16)
    dyd, wd, yd, zd, rd = (t.to(dev) for t in (dy, wp, y0.clone(), z, rb))
    d = L.ConvDesc()
    d.x, d.w, d.y, d.bias = dyd.data_ptr(), wd.data_ptr(), yd.data_ptr(), None
    d.res, d.z = (rd.data_ptr() if res else None), (zd.data_ptr() if dact else None)
    d.x_ld, d.y_ld, d.res_ld, d.z_ld = dy_ld, dx_ld, dx_ld if res else 0, dx_ld if dact else 0
    d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, oh, ow, cout, kpad, 4 * cin
    d.oh, d.ow, d.sy, d.sx = oh, ow, 1, 1
    d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = 2, 2, 0, 0, 1, 1
    d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = H, W, 2, 2, 0, 0
    d.act, d.dact, d.beta, d.dtype, d.out_f32 = 0, (L.ACT_LRELU if dact else 0), int(beta), L.BF16, 0
    d.alpha, d.phc = 0.2, cin
    lib.dvie_trace_kernels(1)
    L.check(lib.dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(L.stream_ptr(dev))), "conv s2 dgrad")
    torch.cuda.synchronize()
    names = lib.dvie_traced_kernels().decode()
    lib.dvie_trace_kernels(0)
    assert names.count("conv_halo_kernel") == 1 and "true>" in names, names
    xs = torch.zeros((n, cin, H, W), requires_grad=True)
    y = F.conv2d(xs, w.float(), stride=2, padding=1)
    (ref,) = torch.autograd.grad(y, xs, dy[..., :cout].float().permute(0, 3, 1, 2))
    if res:
        ref = ref + rb[..., :cin].float().permute(0, 3, 1, 2)
    if beta:
        ref = ref + y0[..., :cin].float().permute(0, 3, 1, 2)
    if dact:
        ref = ref * torch.where(z[..., :cin].float().permute(0, 3, 1, 2) > 0, 1.0, 0.2)
    got = yd.cpu()
    e = rel_l2(got[..., :cin].float().permute(0, 3, 1, 2), ref)
    print(f"s2 dgrad one launch n{n} dx {H}x{W} {cout}->{cin}: rel L2 {e:.2e} ({names})")
    assert e < 4e-3, e
    assert torch.equal(got[..., cin:], y0[..., cin:])  # channels past cin untouched
