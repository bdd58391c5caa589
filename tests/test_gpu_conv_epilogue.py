"""Conv epilogue operands through the C ABI (dvie_conv2d_fwd), every combination of
residual / accumulate (beta) / activation / activation derivative, on the kernels the
library picks by shape: weight-stationary 3x3 (c, cout <= 64, >= 65536 output pixels),
the chunked halo kernel (128- and 64-channel output tiles), the dense-K kernel (c <= 24)
and the 1x1 GEMM (tiled and persistent).  Ragged output sizes put lanes past the image edge in every tile row.

Reference: bf16-rounded operands, conv in fp32 (torch CPU), the same epilogue order
(acc + bias + res + y_old -> act -> dact(z)); tolerance 1e-2 relative to max |y| (bf16
output rounding, fp32 accumulation)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from deep_video_interpolation_extrapolation_amd import _lib as L

pytestmark = pytest.mark.gpu

SHAPES = [  # n, H, W, c, cout, k
    (2, 131, 250, 64, 64, 3),   # conv_ws
    (1, 67, 200, 32, 32, 3),    # conv_ws is skipped below 65536 px: halo cfg 2
    (2, 35, 90, 128, 128, 3),   # halo 128-channel tiles
    (2, 35, 90, 256, 64, 3),    # halo 64-channel tiles, 4 chunks
    (2, 40, 70, 16, 64, 3),     # dense-K
    (2, 37, 77, 128, 256, 1),   # 1x1
    (2, 37, 77, 64, 256, 1),    # 1x1 single K-step, 64-pixel x 128-channel wave tiles: one operand prefetched
    (2, 37, 77, 64, 64, 1),     # 1x1 single K-step, every operand prefetched
    (2, 37, 77, 48, 128, 1),    # 1x1 single K-step, 48 input channels (zero-padded K)
    (2, 37, 77, 32, 96, 1),     # 1x1 single K-step, 32 input channels, partial 64-channel column tile
    (1, 33, 65, 64, 256, 1),    # 1x1 single K-step, ragged pixel count
    (4, 128, 160, 128, 256, 1),  # 1x1 several K-steps, more tiles than resident workgroups: persistent
    (4, 128, 160, 256, 64, 1),   # the same, 64-channel tiles (3-stage ring)
    (3, 131, 177, 192, 96, 1),   # the same, ragged pixel count, partial 128-channel tile
]
MODES = ["none", "res", "beta", "z", "res+z", "beta+z", "res+beta+z"]


def _bf(t):
    return t.to(torch.bfloat16).float()


def _lrelu(v):
    return torch.where(v > 0, v, 0.2 * v)


def _run(dev, shape, mode, out_f32=False, ret_out=False):
    n, H, W, c, cout, k = shape
    g = torch.Generator().manual_seed(7)
    x = _bf(torch.randn(n, H, W, c, generator=g))
    wt = _bf(torch.randn(cout, c, k, k, generator=g) / (c * k * k) ** 0.5)
    bias = torch.randn(cout, generator=g) * 0.1
    res = _bf(torch.randn(n, H, W, cout, generator=g)) if "res" in mode else None
    yold = _bf(torch.randn(n, H, W, cout, generator=g)) if "beta" in mode else None
    z = _bf(torch.randn(n, H, W, cout, generator=g)) if "z" in mode else None
    act = L.ACT_LRELU if mode in ("none", "res", "beta") else L.ACT_NONE

    ref = F.conv2d(x.permute(0, 3, 1, 2), wt, bias, padding=k // 2).permute(0, 2, 3, 1)
    if res is not None:
        ref = ref + res
    if yold is not None:
        ref = ref + yold
    if act == L.ACT_LRELU:
        ref = _lrelu(ref)
    if z is not None:
        ref = ref * torch.where(z > 0, 1.0, 0.2)

    K = k * k * c
    kpad = (K + 63) // 64 * 64
    wp = torch.zeros(cout, kpad)
    wp[:, :K] = wt.permute(0, 2, 3, 1).reshape(cout, K)  # [co][tap * c + ci]
    odt = torch.float32 if out_f32 else torch.bfloat16  # output (and residual) dtype
    xd = x.to(torch.bfloat16).to(dev)
    wd = wp.to(torch.bfloat16).to(dev)
    bd = bias.to(dev)
    yd = (yold if yold is not None else torch.zeros(n, H, W, cout)).to(odt).to(dev)
    rd = res.to(odt).to(dev) if res is not None else None
    zd = z.to(torch.bfloat16).to(dev) if z is not None else None

    d = L.ConvDesc()
    d.x, d.w, d.y, d.bias = xd.data_ptr(), wd.data_ptr(), yd.data_ptr(), bd.data_ptr()
    d.res = rd.data_ptr() if rd is not None else None
    d.z = zd.data_ptr() if zd is not None else None
    d.x_ld, d.y_ld, d.res_ld, d.z_ld = c, cout, cout, cout
    d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, H, W, c, kpad, cout
    d.oh, d.ow, d.sy, d.sx = H, W, 1, 1
    d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = k, k, -(k // 2), -(k // 2), 1, 1
    d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = H, W, 1, 1, 0, 0
    d.act, d.dact, d.beta = act, L.ACT_LRELU if z is not None else L.ACT_NONE, int(yold is not None)
    d.dtype, d.out_f32, d.alpha = L.BF16, int(out_f32), 0.2
    L.check(L.load().dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
            "conv")
    torch.cuda.synchronize()
    out = yd.float().cpu()
    err = float((out - ref).abs().max() / ref.abs().max())
    return (err, out) if ret_out else err


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", SHAPES)
def test_conv_epilogue_operands(dev, shape, mode):
    err = _run(dev, shape, mode)
    assert err < 1e-2, (shape, mode, err)


NK_SHAPES = [  # 3x3 dense-K (c <= 24): the seg head's data-gradient shape and the stems, ragged
    (2, 35, 90, 24, 448, 3),    # 7 output blocks of 64
    (1, 37, 70, 8, 448, 3),
    (2, 40, 70, 16, 64, 3),
    (1, 9, 33, 24, 96, 3),      # one tile per output block, a partial block
]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", NK_SHAPES)
def test_conv_nk_prefetch_bit_exact(dev, shape, mode, monkeypatch):
    """Dense-K kernel with the next tile's epilogue operands prefetched into registers and
    buffer stores (DVIE_NK_PRE=1, the default) against the in-epilogue loads (0): the same
    arithmetic in the same order, so the outputs are equal; both within the fp32 bar."""
    outs = {}
    for pre in ("1", "0"):
        monkeypatch.setenv("DVIE_NK_PRE", pre)
        err, outs[pre] = _run(dev, shape, mode, ret_out=True)
        assert err < 1e-2, (shape, mode, pre, err)
    assert torch.equal(outs["1"], outs["0"]), (shape, mode)


STRIP_SHAPES = [  # 3x3, c and cout <= 64, >= 65536 output pixels: the weight-stationary family
    (2, 131, 250, 64, 64, 3),   # ragged rows (not a multiple of the iteration rows) and columns
    (1, 260, 270, 48, 40, 3),   # 3 K slices, 40 output channels (a partial 32-channel block)
    (8, 20, 2600, 32, 32, 3),   # more strips than resident workgroups: one segment per strip
]


@pytest.mark.parametrize("strip", ["0", "1", "2", "3"])
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", STRIP_SHAPES)
def test_conv_strip_modes(dev, shape, mode, strip, monkeypatch):
    """Strip kernel (DVIE_CONV_STRIP 1-3: rows per iteration / look-ahead) vs the tile kernel
    (0), every epilogue-operand set, bf16 output."""
    monkeypatch.setenv("DVIE_CONV_STRIP", strip)
    err = _run(dev, shape, mode)
    assert err < 1e-2, (shape, mode, strip, err)


NARROW_SHAPES = [  # 3x3, <= 32 output channels from > 64 input channels: conv_narrow.hip
    (2, 35, 90, 448, 24, 3),    # the seg head's channels, ragged rows and columns
    (1, 33, 77, 96, 8, 3),      # the rgb head's padded 8 channels, 3 chunks, partial tiles
    (3, 16, 128, 128, 32, 3),   # a full 32-channel block, 2 tiles per row, more tiles than rows
]


@pytest.mark.parametrize("out_f32", [False, True])
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", NARROW_SHAPES)
def test_conv_narrow_modes(dev, shape, mode, out_f32, monkeypatch):
    """The narrow-output kernel (one step per 32-channel chunk with all 9 taps) and, for
    comparison, the chunked halo kernel it replaces (DVIE_CONV_NARROW=0): every epilogue
    operand set, bf16 and fp32 output."""
    errs = {}
    for env in ("1", "0"):
        monkeypatch.setenv("DVIE_CONV_NARROW", env)
        errs[env] = _run(dev, shape, mode, out_f32=out_f32)
    assert errs["1"] < 1e-2 and errs["0"] < 1e-2, (shape, mode, errs)


@pytest.mark.parametrize("mode", ["none", "res+beta+z"])
@pytest.mark.parametrize("strip", ["0", "1"])
def test_conv_strip_fp32_out(dev, mode, strip, monkeypatch):
    monkeypatch.setenv("DVIE_CONV_STRIP", strip)
    err = _run(dev, (2, 131, 250, 64, 64, 3), mode, out_f32=True)
    assert err < 1e-2, (mode, strip, err)


H8_SHAPES = [  # 3x3, c % 32 == 0, cout % 128 == 0, >= 224 eight-row tiles: conv_h8_kernel
    (4, 125, 250, 128, 128, 3),   # ragged rows and columns, one tile per workgroup
    (8, 61, 120, 256, 256, 3),    # two 128-channel tiles per pixel tile, 8 chunks
    (5, 128, 160, 96, 128, 3),    # 3 chunks of 32 channels
    (3, 200, 256, 128, 128, 3),   # 300 tiles: workgroups run one or two tiles
]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", H8_SHAPES)
def test_conv_h8_modes(dev, shape, mode, monkeypatch):
    """The eight-row halo kernel and, for comparison, the four-row halo kernel it replaces on
    these shapes (DVIE_CONV_H8=0): every epilogue operand set."""
    errs = {}
    for env in ("1", "0"):
        monkeypatch.setenv("DVIE_CONV_H8", env)
        errs[env] = _run(dev, shape, mode)
    assert errs["1"] < 1e-2 and errs["0"] < 1e-2, (shape, mode, errs)


def _run_out(dev, shape, mode):
    """the bf16 output tensor of _run's launch (same seeded operands)"""
    n, H, W, c, cout, k = shape
    g = torch.Generator().manual_seed(7)
    x = _bf(torch.randn(n, H, W, c, generator=g))
    wt = _bf(torch.randn(cout, c, k, k, generator=g) / (c * k * k) ** 0.5)
    bias = torch.randn(cout, generator=g) * 0.1
    res = _bf(torch.randn(n, H, W, cout, generator=g)) if "res" in mode else None
    yold = _bf(torch.randn(n, H, W, cout, generator=g)) if "beta" in mode else None
    z = _bf(torch.randn(n, H, W, cout, generator=g)) if "z" in mode else None
    act = L.ACT_LRELU if mode in ("none", "res", "beta") else L.ACT_NONE
    K = k * k * c
    kpad = (K + 63) // 64 * 64
    wp = torch.zeros(cout, kpad)
    wp[:, :K] = wt.permute(0, 2, 3, 1).reshape(cout, K)
    xd, wd, bd = x.to(torch.bfloat16).to(dev), wp.to(torch.bfloat16).to(dev), bias.to(dev)
    yd = (yold if yold is not None else torch.zeros(n, H, W, cout)).to(torch.bfloat16).to(dev)
    rd = res.to(torch.bfloat16).to(dev) if res is not None else None
    zd = z.to(torch.bfloat16).to(dev) if z is not None else None
    d = L.ConvDesc()
    d.x, d.w, d.y, d.bias = xd.data_ptr(), wd.data_ptr(), yd.data_ptr(), bd.data_ptr()
    d.res = rd.data_ptr() if rd is not None else None
    d.z = zd.data_ptr() if zd is not None else None
    d.x_ld, d.y_ld, d.res_ld, d.z_ld = c, cout, cout, cout
    d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, H, W, c, kpad, cout
    d.oh, d.ow, d.sy, d.sx = H, W, 1, 1
    d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = k, k, -(k // 2), -(k // 2), 1, 1
    d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = H, W, 1, 1, 0, 0
    d.act, d.dact, d.beta = act, L.ACT_LRELU if z is not None else L.ACT_NONE, int(yold is not None)
    d.dtype, d.out_f32, d.alpha = L.BF16, 0, 0.2
    L.check(L.load().dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
            "conv")
    torch.cuda.synchronize()
    return yd.cpu()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", [(2, 37, 77, 64, 256, 1), (1, 33, 65, 64, 256, 1), (4, 64, 128, 64, 256, 1)])
def test_conv_1x1_coalesced_epilogue_bit_exact(dev, shape, mode, monkeypatch):
    """Single-K-step wide 1x1 (64 -> 256): the epilogue whose packed outputs are transposed
    across 8-lane groups before the stores (DVIE_1X1_CE, default) writes the same bits as the
    MFMA-layout stores, ragged last pixel tiles included."""
    out = {}
    for env in ("1", "0"):
        monkeypatch.setenv("DVIE_1X1_CE", env)
        out[env] = _run_out(dev, shape, mode)
    assert torch.equal(out["1"], out["0"]), (shape, mode)

