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
