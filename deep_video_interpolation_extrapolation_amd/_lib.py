"""ctypes binding of libdvie.so (the C ABI declared in include/dvie.h).

The structures below mirror include/dvie.h field for field; `load()` checks every
struct size against `dvie_abi_sizeof` so a header/binding mismatch fails at import.
The library is the only compute path: if it is missing or fails to load, every op
raises — there is no CPU or PyTorch fallback.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (loads torch's HIP runtime first; libdvie reuses it)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdvie.so")

DVIE_OK = 0
DVIE_EINVAL = 1001
F32, BF16 = 0, 1
ACT_NONE, ACT_LRELU, ACT_ELU, ACT_RELU, ACT_TANH = 0, 1, 2, 3, 4
EW_FUSE, EW_UPT, EW_POOL, EW_POOLT, EW_COPY, EW_L1SIGN, EW_NCHW, EW_TONCHW, EW_MASK, EW_IM2COL = range(10)
LOSS_L1, LOSS_GDL, LOSS_SSIM, LOSS_MSE, LOSS_CE, LOSS_L1NHWC, LOSS_COSNHWC, LOSS_IOU, LOSS_ARGMAX_IOU = range(9)
OP_CONV, OP_WGRAD, OP_WREDUCE, OP_COLSUM, OP_EW, OP_LOSS, OP_PACK = 1, 2, 3, 4, 5, 6, 7
OP_BN_FWD, OP_BN_BWD, OP_HEAD_FWD, OP_HEAD_BWD, OP_ATTN, OP_HEAD3_BWD, OP_SEGENC_FWD = 8, 9, 10, 11, 12, 13, 14
OP_SEGENC_BWD = 15
OP_WREDUCE_MULTI = 16
(ATTN_L2NORM, ATTN_L2NORM_BWD, ATTN_CORR, ATTN_GATHER, ATTN_GATHER_T, ATTN_SOFTMAX, ATTN_SOFTMAX_BWD, ATTN_WNORM,
 ATTN_WNORM_BWD, ATTN_POOL, ATTN_POOL_T) = range(11)

vp = ctypes.c_void_p
i32 = ctypes.c_int
i64 = ctypes.c_longlong
f32 = ctypes.c_float


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("x", vp), ("w", vp), ("y", vp), ("bias", vp), ("res", vp), ("z", vp),
        ("x_ld", i64), ("y_ld", i64), ("res_ld", i64), ("z_ld", i64),
        ("n", i32), ("ih", i32), ("iw", i32), ("c", i32),
        ("kpad", i32), ("cout", i32),
        ("oh", i32), ("ow", i32), ("sy", i32), ("sx", i32),
        ("th", i32), ("tw", i32), ("dy0", i32), ("dx0", i32), ("ddy", i32), ("ddx", i32),
        ("yh", i32), ("yw", i32), ("osy", i32), ("osx", i32), ("ory", i32), ("orx", i32),
        ("act", i32), ("dact", i32), ("beta", i32), ("dtype", i32),
        ("out_f32", i32), ("alpha", f32), ("phc", i32), ("pad1", i32),
    ]


class WgradDesc(ctypes.Structure):
    _fields_ = [
        ("g", vp), ("x", vp), ("ws", vp),
        ("g_ld", i64), ("x_ld", i64),
        ("n", i32), ("oh", i32), ("ow", i32), ("cout", i32),
        ("ih", i32), ("iw", i32), ("c", i32), ("sy", i32),
        ("sx", i32), ("th", i32), ("tw", i32), ("dy0", i32),
        ("dx0", i32), ("ddy", i32), ("ddx", i32), ("splits", i32),
        ("dtype", i32), ("tmap", i32), ("bws", vp), ("ws_taps", i32), ("pad1", i32),
    ]


class WreduceDesc(ctypes.Structure):
    _fields_ = [
        ("ws", vp), ("dw", vp), ("cmap", vp),
        ("splits", i32), ("ws_rows", i32), ("ws_k", i32), ("co_off", i32),
        ("cout_p", i32), ("cin_p", i32), ("kh_n", i32), ("kw_n", i32),
        ("c", i32), ("beta", i32),
    ]


class ColsumDesc(ctypes.Structure):
    _fields_ = [
        ("g", vp), ("ws", vp), ("g_ld", i64), ("rows", i64),
        ("c", i32), ("splits", i32), ("dtype", i32), ("pad0", i32),
    ]


class PackDesc(ctypes.Structure):
    _fields_ = [
        ("src", vp), ("dst", vp), ("cmap", vp),
        ("rows", i32), ("kpad", i32), ("c", i32), ("mode", i32),
        ("th", i32), ("tw", i32), ("kh0", i32), ("kw0", i32),
        ("dkh", i32), ("dkw", i32), ("cout_s", i32), ("cin_s", i32),
        ("kh_s", i32), ("kw_s", i32), ("dtype", i32), ("blk0", i32),
    ]


class EwDesc(ctypes.Structure):
    _fields_ = [
        ("y", vp), ("src0", vp), ("src1", vp), ("src2", vp), ("res", vp), ("z", vp),
        ("ext", vp), ("mean", vp), ("std", vp),
        ("y_ld", i64), ("src_ld0", i64), ("src_ld1", i64), ("src_ld2", i64), ("res_ld", i64), ("z_ld", i64),
        ("sn", i64), ("sc", i64), ("sh", i64), ("sw", i64),
        ("op", i32), ("n", i32), ("h", i32), ("w", i32),
        ("c", i32), ("nsrc", i32), ("sh0", i32), ("sw0", i32),
        ("sh1", i32), ("sw1", i32), ("sh2", i32), ("sw2", i32),
        ("act", i32), ("dact", i32), ("beta", i32), ("dtype", i32),
        ("ext_c", i32), ("align", i32),
        ("alpha", f32), ("scale", f32),
    ]


class LossDesc(ctypes.Structure):
    _fields_ = [
        ("a", vp), ("b", vp), ("grad", vp), ("out", vp), ("partial", vp), ("ws", vp),
        ("a_sn", i64), ("a_sc", i64), ("a_sh", i64), ("a_sw", i64),
        ("b_sn", i64), ("b_sc", i64), ("b_sh", i64), ("b_sw", i64),
        ("kind", i32), ("bsz", i32), ("ch", i32), ("h", i32),
        ("w", i32), ("beta", i32), ("dtype", i32), ("out_acc", i32),
        ("weight", f32), ("out_scale", f32),
    ]


class WarpDesc(ctypes.Structure):
    _fields_ = [
        ("img", vp), ("flow", vp), ("out", vp), ("dout", vp), ("dimg", vp), ("dflow", vp), ("ws", vp),
        ("n", i32), ("c", i32), ("h", i32), ("w", i32),
        ("align_corners", i32), ("pad0", i32),
    ]


class ClipDesc(ctypes.Structure):
    _fields_ = [
        ("img", vp), ("seg", vp), ("idx", vp), ("params", vp), ("frames", vp), ("segs", vp), ("bad", vp),
        ("b", i32), ("t", i32), ("h0", i32), ("w0", i32), ("hc", i32), ("wc", i32),
        ("n_classes", i32), ("pad0", i32),
    ]


class BnDesc(ctypes.Structure):
    _fields_ = [
        ("x", vp), ("y", vp), ("g", vp), ("dx", vp), ("gamma", vp), ("beta", vp), ("dgamma", vp), ("dbeta", vp),
        ("running_mean", vp), ("running_var", vp), ("partial", vp), ("stats", vp),
        ("x_ld", i64), ("y_ld", i64), ("g_ld", i64), ("dx_ld", i64), ("rows", i64),
        ("c", i32), ("splits", i32), ("act", i32), ("training", i32),
        ("dtype", i32), ("accumulate", i32), ("beta_dx", i32), ("x_f32", i32),
        ("alpha", f32), ("eps", f32), ("momentum", f32), ("pad1", f32),
    ]


class HeadDesc(ctypes.Structure):
    _fields_ = [
        ("x", vp), ("gx", vp), ("gout", vp), ("out", vp), ("pooled", vp),
        ("x_ld", i64), ("gx_ld", i64),
        ("n", i32), ("h", i32), ("w", i32), ("c", i32),
        ("pool", i32), ("dtype", i32), ("beta", i32), ("pad0", i32),
    ]


class SoftmaxDesc(ctypes.Structure):
    _fields_ = [
        ("x", vp), ("y", vp), ("gy", vp), ("gx", vp),
        ("sn", i64), ("sc", i64), ("sh", i64), ("sw", i64),
        ("n", i32), ("c", i32), ("h", i32), ("w", i32),
        ("beta", i32), ("pad0", i32),
    ]


class SnLayer(ctypes.Structure):
    _fields_ = [
        ("w_bar", vp), ("u", vp), ("v", vp), ("w_eff", vp), ("g_eff", vp), ("g_bar", vp), ("g_u", vp), ("g_v", vp),
        ("state_off", i64),
        ("h", i32), ("width", i32), ("power_iterations", i32), ("beta", i32),
    ]


class AttnDesc(ctypes.Structure):
    _fields_ = [
        ("a", vp), ("b0", vp), ("b1", vp), ("y", vp), ("res", vp), ("z", vp),
        ("a_ld", i64), ("b_ld", i64), ("y_ld", i64), ("res_ld", i64), ("z_ld", i64),
        ("op", i32), ("n", i32), ("h", i32), ("w", i32),
        ("c", i32), ("wh", i32), ("ww", i32), ("nhalf", i32),
        ("half0", i32), ("act", i32), ("dact", i32), ("beta", i32),
        ("dtype", i32), ("pad0", i32),
        ("alpha", f32), ("pad1", f32),
    ]


class PackList(ctypes.Structure):
    _fields_ = [("descs_dev", vp), ("n", i32), ("blocks", i32)]


class Head3BwdDesc(ctypes.Structure):
    _fields_ = [
        ("g", vp), ("h", vp), ("wd", vp), ("dh", vp), ("ws", vp),
        ("g_ld", i64), ("h_ld", i64), ("dh_ld", i64),
        ("n", i32), ("hgt", i32), ("wid", i32), ("c", i32),
        ("cout", i32), ("kpad", i32), ("dy0", i32), ("dx0", i32),
        ("splits", i32), ("dact", i32),
        ("alpha", f32), ("pad0", f32),
    ]


class SegencDesc(ctypes.Structure):
    _fields_ = [
        ("inp", vp), ("e1", vp), ("e2", vp), ("out", vp), ("w0", vp), ("w2", vp), ("w4", vp),
        ("b0", vp), ("b2", vp), ("b4", vp),
        ("in_ld", i64), ("e1_ld", i64), ("e2_ld", i64), ("out_ld", i64),
        ("n", i32), ("h", i32), ("w", i32), ("kpad0", i32), ("kpad2", i32), ("kpad4", i32),
    ]


class SegencBwdDesc(ctypes.Structure):
    _fields_ = [
        ("dout", vp), ("e2", vp), ("e1", vp), ("inp", vp), ("w4d", vp), ("w2d", vp),
        ("dw4", vp), ("dw2", vp), ("dw0", vp), ("db4", vp), ("db2", vp), ("db0", vp),
        ("dout_ld", i64), ("e2_ld", i64), ("e1_ld", i64), ("in_ld", i64),
        ("n", i32), ("h", i32), ("w", i32), ("kpad4", i32), ("kpad2", i32), ("slabs", i32),
    ]


class WreduceMultiDesc(ctypes.Structure):
    """several dvie_wreduce_desc in one launch: `descs` is a HOST array, read at launch time"""
    _fields_ = [("descs", vp), ("n", i32), ("pad", i32)]


class _OpUnion(ctypes.Union):
    _fields_ = [
        ("conv", ConvDesc), ("wgrad", WgradDesc), ("wreduce", WreduceDesc), ("colsum", ColsumDesc),
        ("ew", EwDesc), ("loss", LossDesc), ("pack", PackList), ("bn", BnDesc), ("head", HeadDesc),
        ("attn", AttnDesc), ("head3", Head3BwdDesc), ("segenc", SegencDesc), ("segenc_bwd", SegencBwdDesc),
        ("wreduce_multi", WreduceMultiDesc),
    ]


class Op(ctypes.Structure):
    _fields_ = [("kind", i32), ("lane", i32), ("u", _OpUnion)]


_ABI = {0: Op, OP_CONV: ConvDesc, OP_WGRAD: WgradDesc, OP_WREDUCE: WreduceDesc, OP_COLSUM: ColsumDesc,
        OP_EW: EwDesc, OP_LOSS: LossDesc, OP_PACK: PackDesc, OP_BN_FWD: BnDesc, OP_HEAD_FWD: HeadDesc,
        OP_ATTN: AttnDesc, OP_HEAD3_BWD: Head3BwdDesc, OP_SEGENC_FWD: SegencDesc, OP_SEGENC_BWD: SegencBwdDesc, OP_WREDUCE_MULTI: WreduceMultiDesc, 100: WarpDesc, 101: SoftmaxDesc, 102: SnLayer, 103: ClipDesc}

EXPORTS = [
    "dvie_conv2d_fwd", "dvie_conv2d_wgrad", "dvie_wgrad_splits_hint", "dvie_wgrad_slabs", "dvie_wgrad_reduce", "dvie_wgrad_reduce_multi", "dvie_colsum", "dvie_pack_weights",
    "dvie_ew", "dvie_loss", "dvie_loss_partial_count", "dvie_loss_ws_floats", "dvie_warp_fwd",
    "dvie_warp_bwd", "dvie_adamax", "dvie_scale", "dvie_run_ops", "dvie_abi_sizeof", "dvie_version",
    "dvie_last_error", "dvie_bn_fwd", "dvie_bn_bwd", "dvie_bn_partial_splits", "dvie_head_fwd", "dvie_head_bwd",
    "dvie_softmax_fwd", "dvie_softmax_bwd", "dvie_adam", "dvie_sn_fwd", "dvie_sn_bwd", "dvie_reparam_fwd",
    "dvie_reparam_bwd", "dvie_warp_ws_floats", "dvie_clip_prep", "dvie_attn", "dvie_step_inc", "dvie_adamax_dev",
    "dvie_adam_dev", "dvie_mfma_probe", "dvie_launch_probe", "dvie_sum_f32", "dvie_wgrad_bias_slabs", "dvie_head3_bwd",
    "dvie_segenc_fwd", "dvie_segenc_bwd", "dvie_pack_blocks", "dvie_trace_kernels", "dvie_traced_kernels",
]

_lib = None
_lock = threading.Lock()


class DvieError(RuntimeError):
    pass


def load():
    """Load libdvie.so once; raise loudly if it is absent or its ABI does not match."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DvieError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no non-HIP fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        lib.dvie_abi_sizeof.restype = ctypes.c_size_t
        lib.dvie_abi_sizeof.argtypes = [i32]
        for which, st in _ABI.items():
            got = lib.dvie_abi_sizeof(which)
            if got != ctypes.sizeof(st):
                raise DvieError(f"ABI mismatch for {st.__name__}: C {got} vs ctypes {ctypes.sizeof(st)}")
        lib.dvie_version.restype = ctypes.c_char_p
        lib.dvie_last_error.restype = ctypes.c_char_p
        for name in ("dvie_conv2d_fwd", "dvie_conv2d_wgrad", "dvie_wgrad_reduce", "dvie_colsum", "dvie_ew",
                     "dvie_loss", "dvie_warp_fwd", "dvie_warp_bwd", "dvie_bn_fwd", "dvie_bn_bwd", "dvie_head_fwd",
                     "dvie_head_bwd", "dvie_softmax_fwd", "dvie_softmax_bwd", "dvie_clip_prep", "dvie_attn",
                     "dvie_head3_bwd", "dvie_segenc_fwd", "dvie_segenc_bwd"):
            getattr(lib, name).argtypes = [vp, vp]
            getattr(lib, name).restype = i32
        lib.dvie_pack_weights.argtypes = [vp, i32, i32, vp]
        lib.dvie_wgrad_reduce_multi.argtypes = [vp, i32, vp]
        lib.dvie_wgrad_reduce_multi.restype = i32
        lib.dvie_trace_kernels.argtypes = [i32]
        lib.dvie_trace_kernels.restype = i32
        lib.dvie_traced_kernels.argtypes = []
        lib.dvie_traced_kernels.restype = ctypes.c_char_p
        for name in ("dvie_wgrad_splits_hint", "dvie_wgrad_slabs", "dvie_bn_partial_splits", "dvie_pack_blocks"):
            getattr(lib, name).argtypes = [vp]
            getattr(lib, name).restype = i32
        lib.dvie_run_ops.argtypes = [vp, i32, vp]
        lib.dvie_loss_partial_count.argtypes = [vp]
        lib.dvie_loss_partial_count.restype = ctypes.c_size_t
        lib.dvie_warp_ws_floats.argtypes = [vp]
        lib.dvie_warp_ws_floats.restype = ctypes.c_size_t
        lib.dvie_loss_ws_floats.argtypes = [vp]
        lib.dvie_loss_ws_floats.restype = ctypes.c_size_t
        lib.dvie_adamax.argtypes = [vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, vp]
        lib.dvie_scale.argtypes = [vp, i64, f32, vp]
        lib.dvie_adam.argtypes = [vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, vp]
        f64 = ctypes.c_double
        lib.dvie_adamax_dev.argtypes = [vp, vp, vp, vp, i64, f64, f64, f64, f64, f64, vp, vp]
        lib.dvie_adam_dev.argtypes = [vp, vp, vp, vp, i64, f64, f64, f64, f64, f64, vp, vp]
        lib.dvie_step_inc.argtypes = [vp, vp]
        lib.dvie_mfma_probe.argtypes = [vp, i32, i32, vp]
        lib.dvie_mfma_probe.restype = i32
        lib.dvie_launch_probe.argtypes = [i32, i32, vp]
        lib.dvie_launch_probe.restype = i32
        lib.dvie_sum_f32.argtypes = [vp, i32, vp, vp]
        lib.dvie_sum_f32.restype = i32
        lib.dvie_wgrad_bias_slabs.argtypes = [vp]
        lib.dvie_wgrad_bias_slabs.restype = i32
        for name in ("dvie_sn_fwd", "dvie_sn_bwd"):
            getattr(lib, name).argtypes = [vp, i32, vp, vp]
            getattr(lib, name).restype = i32
        lib.dvie_reparam_fwd.argtypes = [vp, vp, vp, vp, i64, vp]
        lib.dvie_reparam_bwd.argtypes = [vp, vp, vp, vp, vp, i64, i32, vp]
        lib.dvie_reparam_fwd.restype = lib.dvie_reparam_bwd.restype = i32
        _lib = lib
        return lib


def check(rc, what=""):
    if rc != DVIE_OK:
        msg = load().dvie_last_error().decode(errors="replace") if rc == DVIE_EINVAL else f"hipError {rc}"
        raise DvieError(f"{what}: {msg}")


def stream_ptr(device=None):
    """Raw hipStream_t of torch's current stream."""
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(t):
    if not t.is_cuda:
        raise DvieError("dvie ops run on the MI355X only: tensor is on %s (no CPU fallback)" % t.device)
