"""Pointwise multi-resolution ops through the C ABI (dvie_ew) against torch on the same
bf16-rounded operands: EW_FUSE (bilinear upsample of up to three sources, summed, LeakyReLU)
vs F.interpolate (nets/HRNet.py:219-222,577-580), and EW_UPT (the gather-form adjoint of that
upsample) vs autograd through F.interpolate, for 2x / 4x / 8x ratios, both align_corners
modes, ragged sizes and channel slices of wider buffers.  fp32 accumulation in both, bf16
output rounding: tolerance 1e-2 relative to max |y|."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from deep_video_interpolation_extrapolation_amd import _lib as L

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _run(d):
    L.check(L.load().dvie_ew(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "ew")
    torch.cuda.synchronize()


def _desc(op, n, h, w, c, y, y_ld):
    d = L.EwDesc()
    d.op, d.n, d.h, d.w, d.c = op, n, h, w, c
    d.y, d.y_ld = y.data_ptr(), y_ld
    d.dtype, d.alpha, d.scale = L.BF16, 0.2, 1.0
    return d


# (n, fine h, fine w, coarse h, coarse w, c, align)
CASES = [(2, 64, 128, 16, 32, 64, 0), (2, 64, 128, 32, 64, 32, 0), (1, 77, 131, 10, 17, 16, 0),
         (2, 64, 128, 16, 32, 64, 1), (1, 40, 72, 20, 36, 24, 1), (1, 96, 64, 12, 8, 8, 0)]


@pytest.mark.parametrize("case", CASES)
def test_upsample_adjoint(dev, case):
    n, H, W, h, w, c, align = case
    g = torch.Generator().manual_seed(3)
    gy = _bf(torch.randn(n, H, W, c, generator=g))
    x = torch.zeros(n, c, h, w, requires_grad=True)
    F.interpolate(x, size=(H, W), mode="bilinear", align_corners=bool(align)).backward(gy.permute(0, 3, 1, 2))
    ref = x.grad.permute(0, 2, 3, 1)
    # output into a channel slice of a wider buffer, source from one
    yb = torch.zeros(n, h, w, c + 16, dtype=torch.bfloat16, device=dev)
    sb = torch.zeros(n, H, W, c + 8, dtype=torch.bfloat16, device=dev)
    sb[..., 8:] = gy.to(torch.bfloat16)
    d = _desc(L.EW_UPT, n, h, w, c, yb[..., 16:], c + 16)
    d.nsrc, d.src0, d.src_ld0, d.sh0, d.sw0, d.align = 1, sb[..., 8:].data_ptr(), c + 8, H, W, align
    _run(d)
    out = yb[..., 16:].float().cpu()
    err = float((out - ref).abs().max() / ref.abs().max())
    assert err < 1e-2, (case, err)


@pytest.mark.parametrize("pairs", ["1", "0"])
@pytest.mark.parametrize("case", CASES)
def test_fuse_upsample(dev, case, pairs, monkeypatch):
    """EW_FUSE with two output pixels per thread (default) and one (DVIE_EW_FUSE2=0)."""
    monkeypatch.setenv("DVIE_EW_FUSE2", pairs)
    n, H, W, h, w, c, align = case
    g = torch.Generator().manual_seed(5)
    x0 = _bf(torch.randn(n, H, W, c, generator=g))
    x1 = _bf(torch.randn(n, h, w, c, generator=g))
    x2 = _bf(torch.randn(n, max(1, h // 2), max(1, w // 2), c, generator=g))
    ref = x0.clone()
    for s in (x1, x2):
        ref = ref + F.interpolate(s.permute(0, 3, 1, 2), size=(H, W), mode="bilinear",
                                  align_corners=bool(align)).permute(0, 2, 3, 1)
    ref = torch.where(ref > 0, ref, 0.2 * ref)
    y = torch.zeros(n, H, W, c, dtype=torch.bfloat16, device=dev)
    srcs = [t.to(torch.bfloat16).to(dev) for t in (x0, x1, x2)]
    d = _desc(L.EW_FUSE, n, H, W, c, y, c)
    d.nsrc, d.align, d.act = 3, align, L.ACT_LRELU
    for i, t in enumerate(srcs):
        setattr(d, f"src{i}", t.data_ptr())
        setattr(d, f"src_ld{i}", c)
        setattr(d, f"sh{i}", t.shape[1])
        setattr(d, f"sw{i}", t.shape[2])
    _run(d)
    err = float((y.float().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 1e-2, (case, err)


R_CASES = [(2, 64, 128, 16, 32, 64), (2, 64, 128, 32, 64, 32), (1, 48, 80, 12, 20, 256), (1, 40, 72, 20, 36, 128)]


@pytest.mark.parametrize("case", R_CASES)
def test_fuse_single_source_integer_ratio(dev, case, monkeypatch):
    """EW_FUSE of ONE source upsampled 2x / 4x (HRNet's concat and fuse upsamples) on
    ew_fuser_kernel (R outputs per thread), into a channel slice of a wider buffer with an
    accumulate + LeakyReLU-derivative epilogue: equal to ew_fuse2_kernel's result bit for bit
    (same lerp arithmetic per output) and to torch within the bf16 bar."""
    n, H, W, h, w, c = case
    g = torch.Generator().manual_seed(9)
    x1 = _bf(torch.randn(n, h, w, c, generator=g))
    y0 = _bf(torch.randn(n, H, W, c, generator=g))
    z = _bf(torch.randn(n, H, W, c, generator=g))
    ref = F.interpolate(x1.permute(0, 3, 1, 2), size=(H, W), mode="bilinear", align_corners=False).permute(0, 2, 3, 1)
    ref = (ref + y0) * torch.where(z > 0, 1.0, 0.2)
    outs = {}
    for tag, env in (("r", "2"), ("pair", "0")):
        monkeypatch.setenv("DVIE_EW_FUSER", env)
        yb = torch.zeros(n, H, W, c + 24, dtype=torch.bfloat16, device=dev)
        yb[..., 8:8 + c] = y0.to(torch.bfloat16)
        src = x1.to(torch.bfloat16).to(dev)
        zd = z.to(torch.bfloat16).to(dev)
        d = _desc(L.EW_FUSE, n, H, W, c, yb[..., 8:], c + 24)
        d.nsrc, d.align, d.beta, d.dact, d.z, d.z_ld = 1, 0, 1, L.ACT_LRELU, zd.data_ptr(), c
        d.src0, d.src_ld0, d.sh0, d.sw0 = src.data_ptr(), c, h, w
        L.load().dvie_trace_kernels(1)
        _run(d)
        names = L.load().dvie_traced_kernels().decode()
        L.load().dvie_trace_kernels(0)
        assert ("ew_fuser_kernel" in names) == (tag == "r"), names
        outs[tag] = yb.cpu()
    assert torch.equal(outs["r"], outs["pair"])
    got = outs["r"][..., 8:8 + c].float()
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err < 1e-2, (case, err)
    assert not bool(outs["r"][..., :8].any()) and not bool(outs["r"][..., 8 + c:].any())


@pytest.mark.parametrize("c", [24, 40])
@pytest.mark.parametrize("norm", [False, True])
def test_nchw_pack(dev, norm, c):
    """EW_NCHW: fp32 NCHW planes (ext_c of c channels, optional (x - mean) / std as
    preprocess_norm, utils/net_utils.py:11-23) into a bf16 NHWC channel slice; zero channels
    past ext_c.  c <= 32 loads every plane before the first store, c = 40 takes the 8-channel
    loop."""
    n, ec, H, W = 2, 6, 37, 301
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, ec, H, W, generator=g)
    mean = torch.tensor([0.4, 0.5, 0.6, 0.1, 0.2, 0.3] + [0.0] * 2)
    std = torch.tensor([0.2, 0.3, 0.25, 1.0, 0.5, 2.0] + [1.0] * 2)
    ref = torch.zeros(n, H, W, c)
    xr = (x - mean[:ec, None, None]) / std[:ec, None, None] if norm else x
    ref[..., :ec] = xr.permute(0, 2, 3, 1)
    buf = torch.full((n, H, W, c + 8), 7.0, dtype=torch.bfloat16, device=dev)
    xd, md, sd = x.to(dev), mean.to(dev), std.to(dev)
    d = _desc(L.EW_NCHW, n, H, W, c, buf[..., 8:], c + 8)
    d.ext, d.ext_c = xd.data_ptr(), ec
    d.sn, d.sc, d.sh, d.sw = ec * H * W, H * W, W, 1
    if norm:
        d.mean, d.std = md.data_ptr(), sd.data_ptr()
    _run(d)
    out = buf.float().cpu()
    assert float((out[..., 8:] - ref).abs().max()) <= 2e-2 * float(ref.abs().max())
    assert bool((out[..., :8] == 7.0).all()), "write outside the channel slice"


@pytest.mark.parametrize("shape", [(70001, 64, 72, 37), (5000, 24, 24, 7), (131072, 448, 448, 64), (999, 8, 16, 3)])
def test_colsum(dev, shape):
    """dvie_colsum (bias gradients: per-channel column sums of a bf16 [rows][c] gradient with
    row pitch ld, split into `splits` row ranges of fp32 partials) vs torch in fp64."""
    rows, c, ld, splits = shape
    g = torch.Generator().manual_seed(13)
    gb = torch.randn(rows, ld, generator=g).to(torch.bfloat16)
    ref = gb[:, :c].double().sum(0)
    gd = gb.to(dev)
    ws = torch.zeros(splits, c, dtype=torch.float32, device=dev)
    d = L.ColsumDesc()
    d.g, d.ws, d.g_ld, d.rows, d.c, d.splits, d.dtype = gd.data_ptr(), ws.data_ptr(), ld, rows, c, splits, L.BF16
    L.check(L.load().dvie_colsum(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "colsum")
    torch.cuda.synchronize()
    out = ws.double().sum(0).cpu()
    assert float((out - ref).abs().max()) <= 1e-4 * float(ref.abs().max()) + 1e-3
