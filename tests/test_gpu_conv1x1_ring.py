"""GPU: the wide multi-K-step 1x1 convolution on the five-slot operand ring
(conv1x1_ring_kernel, csrc/conv1x1.hip; the heads' 448 -> 896 forward, reference
nets/HRNet.py:410-442 / 584-588) through the C ABI (dvie_conv2d_fwd), against torch's fp32
1x1 conv on the same bf16 operands: ragged pixel counts (tiles past the last pixel), output
channels that are not a multiple of the 256-channel tile, K-steps past the ring's depth,
bias / no bias, LeakyReLU / identity, a channel slice of a wider input (x_ld > c).  Bar: 4e-3
relative L2 (bf16 output rounding); channels past cout untouched; the launch trace names the
kernel."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


CASES = [  # n, h, w, c, x_ld, cout, y_ld, bias, act
    (2, 128, 256, 448, 448, 896, 896, True, True),
    (2, 130, 257, 448, 512, 296, 304, True, False),
    (2, 192, 320, 192, 192, 256, 256, False, True),
    (1, 128, 272, 896, 896, 448, 448, True, True),
]


@pytest.mark.parametrize("n,h,w,c,x_ld,cout,y_ld,bias,act", CASES)
def test_conv1x1_ring_matches_torch(dev, n, h, w, c, x_ld, cout, y_ld, bias, act):
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(c + cout + h)
    xb = torch.randn((n, h, w, x_ld), generator=g).to(torch.bfloat16)
    wt = (torch.randn((cout, c), generator=g) * (1.0 / c) ** 0.5).to(torch.bfloat16)
    bs = torch.randn((cout,), generator=g) * 0.1
    kpad = (c + 63) // 64 * 64
    wp = torch.zeros((cout, kpad), dtype=torch.bfloat16)
    wp[:, :c] = wt
    y0 = torch.randn((n, h, w, y_ld), generator=g).to(torch.bfloat16)  # sentinel contents
    xd, wd, bd, yd = (t.to(dev) for t in (xb, wp, bs, y0.clone()))
    d = L.ConvDesc()
    d.x, d.w, d.y = xd.data_ptr(), wd.data_ptr(), yd.data_ptr()
    d.bias = bd.data_ptr() if bias else None
    d.res, d.z = None, None
    d.x_ld, d.y_ld, d.res_ld, d.z_ld = x_ld, y_ld, 0, 0
    d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, h, w, c, kpad, cout
    d.oh, d.ow, d.sy, d.sx = h, w, 1, 1
    d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = 1, 1, 0, 0, 1, 1
    d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = h, w, 1, 1, 0, 0
    d.act, d.dact, d.beta, d.dtype, d.out_f32 = (L.ACT_LRELU if act else L.ACT_NONE), 0, 0, L.BF16, 0
    d.alpha = 0.2
    lib.dvie_trace_kernels(1)
    L.check(lib.dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(L.stream_ptr(dev))), "conv 1x1 ring")
    torch.cuda.synchronize()
    names = lib.dvie_traced_kernels().decode()
    lib.dvie_trace_kernels(0)
    assert "conv1x1_ring_kernel" in names, names
    ref = xb[..., :c].float().reshape(-1, c) @ wt.float().t()
    if bias:
        ref = ref + bs
    if act:
        ref = F.leaky_relu(ref, 0.2)
    got = yd.cpu()
    out = got[..., :cout].float().reshape(-1, cout)
    e = float((out.double() - ref.double()).norm() / ref.double().norm())
    print(f"ring 1x1 n{n} {h}x{w} {c}->{cout}: rel L2 {e:.2e} ({names})")
    assert e < 4e-3, e
    assert torch.equal(got[..., cout:], y0[..., cout:])  # channels past cout untouched
