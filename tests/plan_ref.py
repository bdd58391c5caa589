"""Descriptor-level reference interpreter of the dvie op lists (test infrastructure only).

Every op a compiled Plan executes is a descriptor whose meaning include/dvie.h states (the
implicit-GEMM conv with its tap grid, output placement and epilogue; the weight-gradient
slabs and their reduction; the pointwise family; the fused head / seg-encoder backwards;
the weight pack).  `Interp` evaluates one descriptor in float64 torch arithmetic on the
very operands the kernel reads -- the plan's stored bf16 activations, its packed bf16
weights, its fp32 slabs -- and either

* checks the kernel's result (`Checker`, the GPU layer-local parity test
  tests/test_gpu_layers.py: the op's output after the launch against the reference, and
  every byte of the output's buffer outside the op's region unchanged), or
* writes the reference result itself (`Executor`: the interpreter runs a whole plan on the
  CPU; tests/test_plan_ref_cpu.py pins the interpreter to the fp64 oracle that way).

Pointers resolve through a registry of the tensors the plan (and the caller) own; a pointer
outside it (an external GPU tensor) is wrapped through __cuda_array_interface__.
The reference semantics follow the reference's ops: nn.Conv2d forward / backward
(nets/HRNet.py, nets/vgg.py), F.interpolate bilinear (nets/HRNet.py:212-225, 576-582),
AvgPool2d (nets/vgg.py:9), the feature L1 (losses.py:178-179).
"""
import ctypes

import torch
import torch.nn.functional as F

from deep_video_interpolation_extrapolation_amd import _lib as L

ACC = torch.float64


def _tdt(code):
    return torch.bfloat16 if code == L.BF16 else torch.float32


def _es(dt):
    return torch.empty((), dtype=dt).element_size()


def act_fwd(v, act, alpha):
    if act == L.ACT_LRELU:
        return torch.where(v > 0, v, v * alpha)
    if act == L.ACT_ELU:
        return torch.where(v > 0, v, torch.expm1(v))
    if act == L.ACT_RELU:
        return torch.where(v > 0, v, torch.zeros_like(v))
    if act == L.ACT_TANH:
        return torch.tanh(v)
    return v


def act_dz(z, act, alpha):
    if act == L.ACT_LRELU:
        return torch.where(z > 0, torch.ones_like(z), torch.full_like(z, alpha))
    if act == L.ACT_ELU:
        return torch.where(z > 0, torch.ones_like(z), z + 1)
    if act == L.ACT_RELU:
        return (z > 0).to(z.dtype)
    if act == L.ACT_TANH:
        return 1 - z * z
    return torch.ones_like(z)


class _CAI:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = dict(shape=(nbytes,), typestr="|u1", data=(ptr, False), version=2)


class Memory:
    """raw pointer -> torch view through registered tensors' storages."""

    def __init__(self, device):
        self.device = device
        self.stores = {}  # storage start -> (end, uint8 tensor over the storage)
        self.snaps = {}  # storage start -> uint8 clone taken before the op

    def add(self, *ts):
        for t in ts:
            if t is None or not isinstance(t, torch.Tensor):
                continue
            st = t.untyped_storage()
            s, n = st.data_ptr(), st.nbytes()
            if n == 0 or s in self.stores:
                continue
            u8 = torch.empty(0, dtype=torch.uint8, device=t.device).set_(st)
            self.stores[s] = (s + n, u8)

    def add_plan(self, plan):
        for b in plan.g.buffers:
            self.add(b.t, b.g)
        self.add(*plan.keep)
        for lay in plan.g.layers:
            self.add(getattr(lay, "wf", None), getattr(lay, "bias_p", None), getattr(lay, "cmap_t", None))
            for _, phases in getattr(lay, "wd", []):
                self.add(*[t for _, t, _ in phases])

    def find(self, ptr, nbytes=1):
        for s, (e, u8) in self.stores.items():
            if s <= ptr and ptr + nbytes <= e:
                return s, u8
        if self.device.type != "cuda":
            raise KeyError(f"pointer {ptr:#x} (+{nbytes}) is in no registered tensor")
        u8 = torch.as_tensor(_CAI(ptr, nbytes), device=self.device)
        self.stores[ptr] = (ptr + nbytes, u8)
        return ptr, u8

    @staticmethod
    def extent(shape, strides):
        return 1 + sum((n - 1) * s for n, s in zip(shape, strides)) if all(shape) else 0

    def view(self, ptr, shape, strides, dt):
        """tensor view of `shape` / element `strides` at ptr"""
        es = _es(dt)
        nb = self.extent(shape, strides) * es
        s, u8 = self.find(ptr, max(1, nb))
        off = ptr - s
        assert off % es == 0, (ptr, dt)
        n = u8.numel() - u8.numel() % es
        typed = u8[:n].view(dt)
        return torch.as_strided(typed, shape, strides, off // es)

    def snapshot(self, ptr):
        s, u8 = self.find(ptr)
        if s not in self.snaps:
            self.snaps[s] = u8.clone()

    def region_bytes(self, ptr, shape, strides, dt):
        """(storage start, byte view of the region) for the unchanged-outside check."""
        es = _es(dt)
        s, u8 = self.find(ptr, max(1, self.extent(shape, strides) * es))
        off = ptr - s
        return s, torch.as_strided(u8, tuple(shape) + (es,), tuple(st * es for st in strides) + (1,), off)

    def clear_snaps(self):
        self.snaps = {}


def nhwc(n, h, w, ld, c):
    return (n, h, w, c), (h * w * ld, w * ld, ld, 1)


class Interp:
    """Reference semantics of each descriptor kind.  Each `ref_*` returns a list of
    (name, ptr, shape, strides, dtype, expected, kind) outputs; kind 'act' = a stored
    activation / gradient (bf16 rounding bar), 'f32' = an fp32 result, 'exact' = bit-exact
    (weight packing), 'slab' = fp32 partial sums (compared as their sum over slabs)."""

    def __init__(self, mem, lib=None):
        self.mem = mem
        self.lib = lib or L.load()

    def rd(self, ptr, shape, strides, dt):
        """an operand, read before the op runs (the reference is evaluated first)"""
        return self.mem.view(ptr, shape, strides, dt).to(ACC)

    # ---------------- convolution ----------------
    def taps_patches(self, x, n_out_h, n_out_w, sy, sx, dys, dxs):
        """x: (n, c, ih, iw) -> {(i, j): (n, c, oh, ow) patch at tap offset (dys[i], dxs[j])}"""
        ih, iw = x.shape[2], x.shape[3]
        top, left = max(0, -min(dys)), max(0, -min(dxs))
        bottom = max(0, (n_out_h - 1) * sy + max(dys) - (ih - 1))
        right = max(0, (n_out_w - 1) * sx + max(dxs) - (iw - 1))
        xp = F.pad(x, (left, right, top, bottom))
        out = {}
        for i, dy in enumerate(dys):
            for j, dx in enumerate(dxs):
                y0, x0 = top + dy, left + dx
                out[(i, j)] = xp[:, :, y0:y0 + (n_out_h - 1) * sy + 1:sy, x0:x0 + (n_out_w - 1) * sx + 1:sx]
        return out

    def conv_acc(self, x_ptr, x_ld, n, ih, iw, c, w_ptr, kpad, cout, oh, ow, sy, sx, th, tw, dy0, dx0, ddy, ddx, dt):
        """acc[n, oy, ox, co] = sum_{t, ci} w[co][t c + ci] x[n][oy sy + dy(t)][ox sx + dx(t)][ci]"""
        x = self.rd(x_ptr, *nhwc(n, ih, iw, x_ld, c), dt).permute(0, 3, 1, 2)
        w = self.rd(w_ptr, (cout, kpad), (kpad, 1), dt)
        dys = [dy0 + i * ddy for i in range(th)]
        dxs = [dx0 + j * ddx for j in range(tw)]
        pt = self.taps_patches(x, oh, ow, sy, sx, dys, dxs)
        acc = torch.zeros((n, oh, ow, cout), dtype=ACC, device=x.device)
        for (i, j), patch in pt.items():
            t = i * tw + j
            acc += torch.einsum("nchw,oc->nhwo", patch, w[:, t * c:(t + 1) * c])
        return acc

    # phase order of dvie_conv_desc.phc (include/dvie.h)
    PH4 = ((0, 0), (1, 1), (0, 1), (1, 0))

    def ref_conv(self, d):
        dt = _tdt(d.dtype)
        ydt = torch.float32 if (d.out_f32 or d.dtype == L.F32) else torch.bfloat16
        v = self.conv_acc(d.x, d.x_ld, d.n, d.ih, d.iw, d.c, d.w, d.kpad, d.cout, d.oh, d.ow, d.sy, d.sx, d.th, d.tw,
                          d.dy0, d.dx0, d.ddy, d.ddx, dt)
        if d.phc:  # one-launch stride-2 data gradient: channel block q -> output phase PH4[q]
            assert d.cout == 4 * d.phc and not d.bias and ydt == torch.bfloat16
            es = _es(ydt)
            out = []
            for q, (a, b) in enumerate(self.PH4):
                oh = min(d.oh, (d.yh - a + 1) // 2)
                ow = min(d.ow, (d.yw - b + 1) // 2)
                if oh <= 0 or ow <= 0:
                    continue
                vq = v[:, :oh, :ow, q * d.phc:(q + 1) * d.phc]

                def at(ptr, ld, a=a, b=b, oh=oh, ow=ow):
                    return (ptr + (a * d.yw + b) * ld * es, (d.n, oh, ow, d.phc),
                            (d.yh * d.yw * ld, 2 * d.yw * ld, 2 * ld, 1))
                if d.res:
                    vq = vq + self.rd(*at(d.res, d.res_ld), ydt)
                yp, ysh, yst = at(d.y, d.y_ld)
                if d.beta:
                    vq = vq + self.rd(yp, ysh, yst, ydt)
                vq = act_fwd(vq, d.act, d.alpha)
                if d.dact:
                    vq = vq * act_dz(self.rd(*at(d.z, d.z_ld), dt), d.dact, d.alpha)
                out.append((f"y phase {a}{b}", yp, ysh, yst, ydt, vq, "act"))
            return out

        def placed(ptr, ld, pdt):
            shape, st = nhwc(d.n, d.oh, d.ow, ld, d.cout)
            st = (d.yh * d.yw * ld, d.osy * d.yw * ld, d.osx * ld, 1)
            return ptr + (d.ory * d.yw + d.orx) * ld * _es(pdt), shape, st

        if d.bias:
            v = v + self.rd(d.bias, (d.cout,), (1,), torch.float32)
        if d.res:
            p, sh, st = placed(d.res, d.res_ld, ydt)
            v = v + self.rd(p, sh, st, ydt)
        yp, ysh, yst = placed(d.y, d.y_ld, ydt)
        if d.beta:
            v = v + self.rd(yp, ysh, yst, ydt)
        v = act_fwd(v, d.act, d.alpha)
        if d.dact:
            p, sh, st = placed(d.z, d.z_ld, dt)
            v = v * act_dz(self.rd(p, sh, st, dt), d.dact, d.alpha)
        return [("y", yp, ysh, yst, ydt, v, "act" if ydt == torch.bfloat16 else "f32")]

    # ---------------- weight gradient ----------------
    def wgrad_sum(self, g_ptr, g_ld, x_ptr, x_ld, n, oh, ow, cout, ih, iw, c, sy, sx, th, tw, dy0, dx0, ddy, ddx, dt,
                  xw=None):
        """[cout][taps][c]: sum_pix g[pix][co] x[pix + tap][ci]; xw: the number of valid x
        columns when iw is only the row pitch (the stride-2 phase views)"""
        g = self.rd(g_ptr, *nhwc(n, oh, ow, g_ld, cout), dt)
        if xw is None:
            x = self.rd(x_ptr, *nhwc(n, ih, iw, x_ld, c), dt).permute(0, 3, 1, 2)
        else:
            x = self.rd(x_ptr, (n, ih, xw, c), (ih * iw * x_ld, iw * x_ld, x_ld, 1), dt).permute(0, 3, 1, 2)
        dys = [dy0 + i * ddy for i in range(th)]
        dxs = [dx0 + j * ddx for j in range(tw)]
        pt = self.taps_patches(x, oh, ow, sy, sx, dys, dxs)
        out = torch.zeros((cout, th * tw, c), dtype=ACC, device=g.device)
        for (i, j), patch in pt.items():
            out[:, i * tw + j] = torch.einsum("nhwo,nchw->oc", g, patch)
        return out, g

    def ref_wgrad(self, d):
        dt = _tdt(d.dtype)
        T = d.th * d.tw
        dw, g = self.wgrad_sum(d.g, d.g_ld, d.x, d.x_ld, d.n, d.oh, d.ow, d.cout, d.ih, d.iw, d.c, d.sy, d.sx, d.th,
                               d.tw, d.dy0, d.dx0, d.ddy, d.ddx, dt, xw=d.ow if d.ws_taps else None)
        slabs = self.lib.dvie_wgrad_slabs(ctypes.byref(d))
        if d.ws_taps:  # a phase launch of a shared slab set: its taps' column blocks only
            K = d.ws_taps * d.c
            out = [(f"dW slabs tap {t} -> {(d.tmap >> 4 * t) & 15}", d.ws + 4 * ((d.tmap >> 4 * t) & 15) * d.c,
                    (slabs, d.cout, d.c), (d.cout * K, K, 1), torch.float32, dw[:, t], "slab") for t in range(T)]
        else:
            out = [("dW slabs", d.ws, (slabs, d.cout, T * d.c), (d.cout * T * d.c, T * d.c, 1), torch.float32,
                    dw.reshape(d.cout, T * d.c), "slab")]
        if d.bws:
            bs = self.lib.dvie_wgrad_bias_slabs(ctypes.byref(d))
            out.append(("db slabs", d.bws, (bs, d.cout), (d.cout, 1), torch.float32, g.sum((0, 1, 2)), "slab"))
        return out

    def ref_wreduce(self, d):
        ws = self.rd(d.ws, (d.splits, d.ws_rows, d.ws_k), (d.ws_rows * d.ws_k, d.ws_k, 1), torch.float32)
        T = d.kh_n * d.kw_n
        S = ws.sum(0)[d.co_off:d.co_off + d.cout_p].reshape(d.cout_p, T, d.c)
        shape = (d.cout_p, d.cin_p, d.kh_n, d.kw_n)
        strides = (d.cin_p * T, T, d.kw_n, 1)
        ref = torch.zeros((d.cout_p, d.cin_p, T), dtype=ACC, device=ws.device)
        cmap = (self.mem.view(d.cmap, (d.c,), (1,), torch.int32).cpu().tolist() if d.cmap else list(range(d.c)))
        for j, ci in enumerate(cmap):
            if 0 <= ci < d.cin_p:
                ref[:, ci] += S[:, :, j]
        ref = ref.reshape(shape)
        if d.beta:
            ref = ref + self.rd(d.dw, shape, strides, torch.float32)
        return [("dW", d.dw, shape, strides, torch.float32, ref, "f32")]

    def ref_colsum(self, d):
        dt = _tdt(d.dtype)
        g = self.rd(d.g, (d.rows, d.c), (d.g_ld, 1), dt)
        return [("colsum slabs", d.ws, (d.splits, d.c), (d.c, 1), torch.float32, g.sum(0), "slab")]

    # ---------------- weight packing ----------------
    def ref_pack_one(self, d):
        src = self.rd(d.src, (d.cout_s, d.cin_s, d.kh_s, d.kw_s), (d.cin_s * d.kh_s * d.kw_s, d.kh_s * d.kw_s, d.kw_s, 1),
                      torch.float32)
        dst_dt = _tdt(d.dtype)
        out = torch.zeros((d.rows, d.kpad), dtype=ACC, device=src.device)
        ntap = d.th * d.tw
        cm = None
        if d.cmap:
            n = d.c if d.mode == 0 else d.rows
            cm = self.mem.view(d.cmap, (n,), (1,), torch.int32).to(torch.long)
        for t in range(ntap):
            kh = d.kh0 + (t // d.tw) * d.dkh
            kw = d.kw0 + (t % d.tw) * d.dkw
            if not (0 <= kh < d.kh_s and 0 <= kw < d.kw_s):
                continue
            s2 = src[:, :, kh, kw]  # [co][ci]
            if d.mode == 0:  # dst[r][t c + j] = src[r][cmap[j]]
                ci = cm if cm is not None else torch.arange(d.c, device=src.device)
                ok = (ci >= 0) & (ci < d.cin_s)
                rr = min(d.rows, d.cout_s)
                blk = torch.zeros((rr, d.c), dtype=ACC, device=src.device)
                blk[:, ok] = s2[:rr][:, ci[ok]]
                out[:rr, t * d.c:(t + 1) * d.c] = blk
            else:  # dst[r][t c + j] = src[j][cmap[r]]
                ci = cm if cm is not None else torch.arange(d.rows, device=src.device)
                ok = (ci >= 0) & (ci < d.cin_s)
                jj = min(d.c, d.cout_s)
                blk = torch.zeros((d.rows, d.c), dtype=ACC, device=src.device)
                blk[ok, :jj] = s2[:jj][:, ci[ok]].t()
                out[:, t * d.c:(t + 1) * d.c] = blk
        return ("pack", d.dst, (d.rows, d.kpad), (d.kpad, 1), dst_dt, out, "exact")

    def ref_pack(self, o, descs):
        return [self.ref_pack_one(d) for d in descs]

    # ---------------- pointwise ----------------
    def ref_ew(self, d):
        dt = _tdt(d.dtype)
        n, h, w, c = d.n, d.h, d.w, d.c
        srcs = [(d.src0, d.src_ld0, d.sh0, d.sw0), (d.src1, d.src_ld1, d.sh1, d.sw1),
                (d.src2, d.src_ld2, d.sh2, d.sw2)]
        dev = self.mem.device

        def src(i, hh=None, ww=None, cc=None):
            p, ld, sh, sw = srcs[i]
            return self.rd(p, *nhwc(n, hh or sh, ww or sw, ld, cc or c), dt)

        op = d.op
        if op == L.EW_TONCHW:
            a = src(0, h, w, c)[..., :d.ext_c].permute(0, 3, 1, 2)
            if d.std:
                a = a / self.rd(d.std, (d.ext_c,), (1,), torch.float32).view(1, -1, 1, 1)
            shape, st = (n, d.ext_c, h, w), (d.sn, d.sc, d.sh, d.sw)
            if d.beta:
                a = a + self.rd(d.ext, shape, st, torch.float32)
            return [("ext", d.ext, shape, st, torch.float32, a, "f32")]
        if op == L.EW_FUSE:
            v = torch.zeros((n, c, h, w), dtype=ACC, device=dev)
            for i in range(d.nsrc):
                s = src(i).permute(0, 3, 1, 2)
                if s.shape[2:] != (h, w):
                    s = F.interpolate(s, size=(h, w), mode="bilinear", align_corners=bool(d.align))
                v = v + s
            v = v.permute(0, 2, 3, 1)
        elif op == L.EW_UPT:
            s = src(0).permute(0, 3, 1, 2)
            x = torch.zeros((n, c, h, w), dtype=ACC, device=dev, requires_grad=True)
            with torch.enable_grad():
                up = F.interpolate(x, size=(d.sh0, d.sw0), mode="bilinear", align_corners=bool(d.align))
                (gx,) = torch.autograd.grad(up, x, s)
            v = gx.permute(0, 2, 3, 1)
        elif op == L.EW_POOL:
            v = F.avg_pool2d(src(0).permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
        elif op == L.EW_POOLT:
            v = src(0).repeat_interleave(2, 1).repeat_interleave(2, 2)[:, :h, :w] / 4
        elif op == L.EW_COPY:
            v = src(0, h, w)
        elif op == L.EW_L1SIGN:
            v = d.scale * torch.sign(src(0, h, w) - src(1, h, w))
        elif op == L.EW_NCHW:
            v = torch.zeros((n, h, w, c), dtype=ACC, device=dev)
            st = (d.sn, d.sc, d.sh, d.sw)
            if d.src1:
                k0 = d.sh1
                v[..., :k0] = self.rd(d.ext, (n, k0, h, w), st, torch.float32).permute(0, 2, 3, 1)
                v[..., k0:d.ext_c] = self.rd(d.src1, (n, d.ext_c - k0, h, w), st, torch.float32).permute(0, 2, 3, 1)
            else:
                v[..., :d.ext_c] = self.rd(d.ext, (n, d.ext_c, h, w), st, torch.float32).permute(0, 2, 3, 1)
            if d.mean:
                m = self.rd(d.mean, (d.ext_c,), (1,), torch.float32)
                s = self.rd(d.std, (d.ext_c,), (1,), torch.float32)
                v[..., :d.ext_c] = (v[..., :d.ext_c] - m) / s
        elif op == L.EW_MASK:
            m = self.rd(d.ext, (n, h, w), (d.sn, d.sh, d.sw), torch.float32)
            f = 1 - m if d.ext_c else m
            v = src(0, h, w) * f.unsqueeze(-1)
        elif op == L.EW_IM2COL:
            p, ld = d.src0, d.src_ld0
            s = self.rd(p, *nhwc(n, h, w, ld, d.ext_c), dt).permute(0, 3, 1, 2)
            v = torch.zeros((n, h, w, c), dtype=ACC, device=dev)
            pt = self.taps_patches(s, h, w, 1, 1, [d.sh1 + i * d.sh2 for i in range(d.sh0)],
                                   [d.sw1 + j * d.sw2 for j in range(d.sw0)])
            for (i, j), patch in pt.items():
                t = i * d.sw0 + j
                v[..., t * d.ext_c:(t + 1) * d.ext_c] = patch.permute(0, 2, 3, 1)
        else:
            raise NotImplementedError(f"ew op {op}")
        shape, st = nhwc(n, h, w, d.y_ld, c)
        if d.res:
            v = v + self.rd(d.res, *nhwc(n, h, w, d.res_ld, c), dt)
        if d.beta:
            v = v + self.rd(d.y, shape, st, dt)
        v = act_fwd(v, d.act, d.alpha)
        if d.dact:
            v = v * act_dz(self.rd(d.z, *nhwc(n, h, w, d.z_ld, c), dt), d.dact, d.alpha)
        return [("y", d.y, shape, st, dt, v, "act" if dt == torch.bfloat16 else "f32")]

    # ---------------- losses inside plans (VGG feature L1) ----------------
    def ref_loss(self, d):
        assert d.kind == L.LOSS_L1NHWC and not d.grad, "only the plan's feature-L1 loss is interpreted"
        dt = _tdt(d.dtype)
        shape = (d.bsz, d.ch, d.h, d.w)
        a = self.rd(d.a, shape, (d.a_sn, d.a_sc, d.a_sh, d.a_sw), dt)
        b = self.rd(d.b, shape, (d.b_sn, d.b_sc, d.b_sh, d.b_sw), dt)
        v = (a - b).abs().mean() * d.out_scale
        if d.out_acc:
            v = v + self.rd(d.out, (1,), (1,), torch.float32)[0]
        return [("loss", d.out, (1,), (1,), torch.float32, v.reshape(1), "f32")]

    # ---------------- fused head backward ----------------
    def ref_head3(self, d):
        dt = torch.bfloat16
        co, c = d.cout, d.c
        # dh: the data-gradient conv over g (co channels) with the packed weights wd [c][kpad]
        v = self.conv_acc(d.g, d.g_ld, d.n, d.hgt, d.wid, co, d.wd, d.kpad, c, d.hgt, d.wid, 1, 1, 3, 3, d.dy0, d.dx0,
                          1, 1, dt)
        hsh, hst = nhwc(d.n, d.hgt, d.wid, d.h_ld, c)
        h = self.rd(d.h, hsh, hst, dt)
        if d.dact:
            v = v * act_dz(h, d.dact, d.alpha)
        # slabs: ws[s][o][(8 - t) c + ci] = sum_p g[p + (dy0 + i_t, dx0 + j_t)][o] h[p][ci]
        g = self.rd(d.g, *nhwc(d.n, d.hgt, d.wid, d.g_ld, co), dt).permute(0, 3, 1, 2)
        pt = self.taps_patches(g, d.hgt, d.wid, 1, 1, [d.dy0 + i for i in range(3)], [d.dx0 + j for j in range(3)])
        ref = torch.zeros((co, 9, c), dtype=ACC, device=g.device)
        for (i, j), patch in pt.items():
            t = 3 * i + j
            ref[:, 8 - t] = torch.einsum("nohw,nhwc->oc", patch, h)
        dsh, dst = nhwc(d.n, d.hgt, d.wid, d.dh_ld, c)
        return [("dh", d.dh, dsh, dst, dt, v, "act"),
                ("dW slabs", d.ws, (d.splits, co, 9 * c), (co * 9 * c, 9 * c, 1), torch.float32, ref.reshape(co, 9 * c),
                 "slab")]

    # ---------------- fused seg-encoder forward ----------------
    def ref_segenc_fwd(self, d):
        """e1 = ELU(conv0(in) + b0), e2 = ELU(conv2(e1) + b2), out = conv4(e2) + b4 (3x3, pad 1),
        e1 / e2 stored bf16 and each conv reading the previous one's bf16 map (the kernel's LDS
        images hold exactly those values)"""
        dt = torch.bfloat16
        n, h, w = d.n, d.h, d.w
        geo = (h, w, 1, 1, 3, 3, -1, -1, 1, 1, dt)
        v = self.conv_acc(d.inp, d.in_ld, n, h, w, 24, d.w0, d.kpad0, 32, *geo)
        e1 = act_fwd(v + self.rd(d.b0, (32,), (1,), torch.float32), L.ACT_ELU, 0.0)
        t1 = self._tmp(e1)
        v = self.conv_acc(t1.data_ptr(), 32, n, h, w, 32, d.w2, d.kpad2, 32, *geo)
        e2 = act_fwd(v + self.rd(d.b2, (32,), (1,), torch.float32), L.ACT_ELU, 0.0)
        t2 = self._tmp(e2)
        out = self.conv_acc(t2.data_ptr(), 32, n, h, w, 32, d.w4, d.kpad4, 8, *geo)
        out = out + self.rd(d.b4, (8,), (1,), torch.float32)
        self._tmps = []
        e1sh, e1st = nhwc(n, h, w, d.e1_ld, 32)
        e2sh, e2st = nhwc(n, h, w, d.e2_ld, 32)
        osh, ost = nhwc(n, h, w, d.out_ld, 8)
        return [("e1", d.e1, e1sh, e1st, dt, e1, "act"), ("e2", d.e2, e2sh, e2st, dt, e2, "act"),
                ("out", d.out, osh, ost, dt, out, "act")]

    # ---------------- fused seg-encoder backward ----------------
    def ref_segenc_bwd(self, d):
        dt = torch.bfloat16
        n, h, w = d.n, d.h, d.w
        e2 = self.rd(d.e2, *nhwc(n, h, w, d.e2_ld, 32), dt)
        e1 = self.rd(d.e1, *nhwc(n, h, w, d.e1_ld, 32), dt)
        # d_e2 = ELU'(e2) conv4^T(dout), d_e1 = ELU'(e1) conv2^T(d_e2), both bf16 on chip
        de2 = self.conv_acc(d.dout, d.dout_ld, n, h, w, 8, d.w4d, d.kpad4, 32, h, w, 1, 1, 3, 3, -1, -1, 1, 1, dt)
        de2 = (de2 * act_dz(e2, L.ACT_ELU, 0.0)).to(dt).to(ACC)
        tmp = self._tmp(de2)
        de1 = self.conv_acc(tmp.data_ptr(), 32, n, h, w, 32, d.w2d, d.kpad2, 32, h, w, 1, 1, 3, 3, -1, -1, 1, 1, dt)
        de1 = (de1 * act_dz(e1, L.ACT_ELU, 0.0)).to(dt).to(ACC)
        tmp1 = self._tmp(de1)
        out = []
        for name, gp, gld, co, xp, xld, ci, wsp, bsp in (
                ("conv4", d.dout, d.dout_ld, 8, d.e2, d.e2_ld, 32, d.dw4, d.db4),
                ("conv2", tmp.data_ptr(), 32, 32, d.e1, d.e1_ld, 32, d.dw2, d.db2),
                ("conv0", tmp1.data_ptr(), 32, 32, d.inp, d.in_ld, 24, d.dw0, d.db0)):
            dw, g = self.wgrad_sum(gp, gld, xp, xld, n, h, w, co, h, w, ci, 1, 1, 3, 3, -1, -1, 1, 1, dt)
            out.append((name + " dW slabs", wsp, (d.slabs, co, 9 * ci), (co * 9 * ci, 9 * ci, 1), torch.float32,
                        dw.reshape(co, 9 * ci), "slab"))
            out.append((name + " db slabs", bsp, (d.slabs, co), (co, 1), torch.float32, g.sum((0, 1, 2)), "slab"))
        self._tmps = []
        return out

    def _tmp(self, v):
        """a bf16 NHWC copy of an on-chip intermediate, addressable by pointer"""
        t = v.to(torch.bfloat16).contiguous()
        self.mem.add(t)
        self._tmps = getattr(self, "_tmps", []) + [t]
        return t

    # ---------------- dispatch ----------------
    def outputs(self, o, plan=None):
        k = o.kind
        if k == L.OP_CONV:
            return self.ref_conv(o.u.conv)
        if k == L.OP_WGRAD:
            return self.ref_wgrad(o.u.wgrad)
        if k == L.OP_WREDUCE:
            return self.ref_wreduce(o.u.wreduce)
        if k == L.OP_WREDUCE_MULTI:  # a batch of reductions: each one's result
            m = o.u.wreduce_multi
            descs = (L.WreduceDesc * m.n).from_address(m.descs)
            return [out for d in descs for out in self.ref_wreduce(d)]
        if k == L.OP_COLSUM:
            return self.ref_colsum(o.u.colsum)
        if k == L.OP_EW:
            return self.ref_ew(o.u.ew)
        if k == L.OP_LOSS:
            return self.ref_loss(o.u.loss)
        if k == L.OP_PACK:
            return self.ref_pack(o, plan._pack_descs)
        if k == L.OP_HEAD3_BWD:
            return self.ref_head3(o.u.head3)
        if k == L.OP_SEGENC_BWD:
            return self.ref_segenc_bwd(o.u.segenc_bwd)
        if k == L.OP_SEGENC_FWD:
            return self.ref_segenc_fwd(o.u.segenc)
        raise NotImplementedError(f"op kind {k}")


def rel_l2(got, ref):
    got, ref = got.to(ACC), ref.to(ACC)
    den = float(ref.norm())
    num = float((got - ref).norm())
    if den == 0.0:
        return 0.0 if num == 0.0 else float("inf")
    return num / den


class Executor:
    """engine.OP_HOOK that runs every op through the interpreter instead of the library
    (CPU plans): slab outputs get the whole sum in slab 0 and zeros elsewhere."""

    def __init__(self, mem):
        self.mem = mem
        self.ip = Interp(mem)
        self.kinds = {}

    def __call__(self, plan, arr, i, meta, run):
        self.mem.add_plan(plan)
        o = arr[i]
        outs = self.ip.outputs(o, plan)
        for name, ptr, shape, strides, dt, v, kind in outs:
            y = self.mem.view(ptr, shape, strides, dt)
            if kind == "slab":
                y.zero_()
                y[0].copy_(v.reshape(y[0].shape).to(dt))
            else:
                y.copy_(v.to(dt))
        self.kinds[o.kind] = self.kinds.get(o.kind, 0) + 1


# bars (relative L2 against the float64 reference of the op's own operands)
BARS = {"act": 4e-3,  # a stored bf16 activation / gradient: the output rounding
        "f32": 1e-4,  # an fp32 result (fp32 accumulation order)
        "slab": 1e-4,  # fp32 weight-gradient / column-sum partials, summed over the slabs
        "exact": 0.0}  # packed weights: bit-exact


class Checker:
    """engine.OP_HOOK for the GPU layer-local parity test: evaluate the reference of each op
    on its operands, snapshot the buffers it writes, launch it (the product kernel, with the
    library's launch trace on), then compare its outputs and check that nothing outside its
    output regions changed.  One record per op: (list, index, kind, layer, kernels, worst
    error, bar, output names)."""

    def __init__(self, mem, lib=None, skip_kinds=()):
        self.mem = mem
        self.lib = lib or L.load()
        self.ip = Interp(mem, self.lib)
        self.records = []
        self.skip_kinds = set(skip_kinds)
        self.failures = []

    def __call__(self, plan, arr, i, meta, run):
        self.mem.add_plan(plan)
        o = arr[i]
        if o.kind in self.skip_kinds:
            run()
            self.records.append(dict(kind=o.kind, name=(meta or {}).get("name", ""), kernels="", err=None, bar=None,
                                     outs=[], checked=False))
            return
        outs = self.ip.outputs(o, plan)
        dev = self.mem.device
        if dev.type == "cuda":
            torch.cuda.synchronize()
        # the buffers this op writes, except the shared slab workspaces (untouched check)
        guarded = {}
        for name, ptr, shape, strides, dt, v, kind in outs:
            if kind == "slab":
                continue
            s, _ = self.mem.region_bytes(ptr, shape, strides, dt)
            if s not in guarded:
                guarded[s] = self.mem.stores[s][1].clone()
        self.lib.dvie_trace_kernels(1)
        run()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        kernels = self.lib.dvie_traced_kernels().decode(errors="replace")
        self.lib.dvie_trace_kernels(0)
        worst, bar_of_worst, names = 0.0, None, []
        for name, ptr, shape, strides, dt, v, kind in outs:
            got = self.mem.view(ptr, shape, strides, dt)
            if kind == "slab":
                got = got.to(ACC).sum(0)
                v = v.reshape(got.shape)
            if kind == "exact":
                err = 0.0 if torch.equal(got, v.to(dt)) else float("inf")
            else:
                err = rel_l2(got, v)
                if not bool(torch.isfinite(got.to(ACC)).all()):
                    err = float("inf")
            names.append(f"{name}:{err:.2e}")
            if err > BARS[kind]:
                self.failures.append((i, o.kind, (meta or {}).get("name", ""), name, err, BARS[kind], kernels))
            if bar_of_worst is None or err / max(BARS[kind], 1e-30) > worst / max(bar_of_worst, 1e-30):
                worst, bar_of_worst = err, BARS[kind]
        # nothing outside the written regions changed
        changed = {s: self.mem.stores[s][1] != snap for s, snap in guarded.items()}
        for name, ptr, shape, strides, dt, v, kind in outs:
            if kind == "slab":
                continue
            s, rb = self.mem.region_bytes(ptr, shape, strides, dt)
            _, cb = s, torch.as_strided(changed[s], rb.shape, rb.stride(), rb.storage_offset())
            cb.zero_()
        for s, ch in changed.items():
            if bool(ch.any()):
                self.failures.append((i, o.kind, (meta or {}).get("name", ""), "outside-region write",
                                      int(ch.sum()), 0, kernels))
        self.records.append(dict(kind=o.kind, name=(meta or {}).get("name", ""), kernels=kernels, err=worst,
                                 bar=bar_of_worst, outs=names, checked=True))
        del outs, guarded, changed


def track(mem, setattr_):
    """Register the external tensors plans are pointed at (inputs, outputs, output / input
    gradients, parameter gradients, loss outputs) as the owners patch them in, so every
    operand pointer resolves through the registry.  setattr_: monkeypatch.setattr."""
    from deep_video_interpolation_extrapolation_amd import engine as E

    def wrap(name, regs):
        orig = getattr(E.Plan, name)

        def f(self, *a, **k):
            out = orig(self, *a, **k)
            mem.add_plan(self)
            for t in regs(self, a, k):
                mem.add(t)
            return out

        setattr_(E.Plan, name, f)

    def tensors(a, k):
        out = []
        for x in list(a) + list(k.values()):
            if isinstance(x, torch.Tensor):
                out.append(x)
            elif isinstance(x, (list, tuple)):
                out += [t for t in x if isinstance(t, torch.Tensor)]
        return out

    for nm in ("set_input", "set_input_parts", "set_output", "set_output_grad", "set_input_grad", "set_output_nchw",
               "set_mask", "set_head_output", "set_head_grad", "set_l1_loss"):
        wrap(nm, lambda self, a, k: tensors(a, k))

    def params(self, a, k):
        out = []
        for lay in self.g.layers:
            m = lay.m
            ps = m.params() if isinstance(m, E.StackedConv) else [m.weight, getattr(m, "bias", None)]
            for p in ps:
                if p is not None:
                    out += [p, p.grad]
        return out

    wrap("set_param_grads", params)
    orig_run = E.Plan.run_forward

    def run_forward(self, *a, **k):  # parameters (the pack's sources)
        mem.add_plan(self)
        for t in params(self, (), {}):
            mem.add(t)
        return orig_run(self, *a, **k)

    setattr_(E.Plan, "run_forward", run_forward)
