"""VAEHRNet (reference nets/HRNet.py:702-1061), the coarse model the reference InterGANNet
unpacks (rgb, seg, mu, logvar) from, on the MI355X plan engine.

Same module tree, construction order (so seeded initialisation) and state_dict keys as the
reference: vae_encoder, mu_fc, logvar_fc, vae_decoder, then the HRNet trunk whose stem takes
46 channels cat([vae_feature(32), input[:, :6], seg_enc(seg1), seg_enc(seg2)]) (l.993-997).
The training forward runs as four plans chained by autograd, all on HIP kernels:

  1. vae_encoder over the packed inputs [x | seg | gt_x | gt_seg] (convs, train-mode
     BatchNorm + LeakyReLU; l.972-973) -> (B, 16, 8, 8);
  2. mu_fc / logvar_fc: the two Linear(1024, 1024) as 1x1 convs over the (B, 1, 1, 1024)
     flattening in the reference's view(-1, 1024) order (l.974-976);
  3. z = eps * exp(0.5 * logvar) + mu (dvie_reparam_fwd; reparameterize l.960-964), eps drawn
     like the reference's std.new(std.size()).normal_() (torch's device generator here);
  4. vae_decoder (ConvTranspose2d(4, 2, 1) as the strided-conv data-gradient phases, BatchNorm,
     LeakyReLU; l.764-791) -> vae_feature (B, 32, H, W);
  5. the HRNet trunk plan with vae_feature packed into the stem buffer.
Eval: z ~ N(0, 1) (l.965-966), decoder, trunk.  Like the reference (view(-1, 1024) of a
16 x H/16 x W/16 code) it only runs at 128 x 128.
"""
import ctypes

import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import PlanFunction, PlanPool
from .conv import Conv2d
from .disc import _packing, lower_sequential
from .HRNet import HRNet


def _cbl(cin, cout, s=1):
    return [Conv2d(cin, cout, 3, s, 1), nn.BatchNorm2d(cout), nn.LeakyReLU(0.2, inplace=True)]


def _tbl(cin, cout):
    return [nn.ConvTranspose2d(cin, cout, 4, stride=2, padding=1), nn.BatchNorm2d(cout),
            nn.LeakyReLU(0.2, inplace=True)]


class _SeqRunner:
    """One nn.Sequential of a FlatParams owner as an engine plan: external NCHW fp32 inputs
    packed into channel slices of the first buffer; the last conv's fp32 map is the output."""

    def __init__(self, owner, seq, prefix, widths, key):
        self.owner, self.seq, self.prefix, self.widths, self.key = owner, seq, prefix, widths, key
        self.params = list(seq.parameters())
        self.pool = PlanPool(self._build)

    def _build(self, pkey):
        n, H, W, dtype, bn_train, trainable, in_grads, backward, dev = pkey
        g = E.Graph(dtype)
        g.bn_training = bn_train
        slices, cmap, total = _packing(self.widths)
        inp = g.buffer(f"{self.prefix}.in", H, W, total)
        for k, (c0, c, w) in enumerate(slices):
            g.input_nchw(E.R(inp, c0, c), f"in{k}", ext_c=w, requires_grad=bool(in_grads[k]))
        if cmap == list(range(total)):
            cmap = None
        lower_sequential(g, list(self.seq), E.R(inp), self.prefix, trainable, cmap=cmap, out_key=self.key)
        return g.compile(n, dev, backward=backward)

    def run_forward(self, inputs, train):
        x = inputs[0]
        L.require_gpu(x)
        n, _, H, W = x.shape
        needs = getattr(self, "_in_needs", (False,) * len(inputs))
        trainable = bool(train) and any(p.requires_grad for p in self.params)
        in_grads = tuple(bool(train) and bool(k) for k in needs)
        backward = trainable or any(in_grads)
        plan = self.pool.acquire((n, H, W, self.owner.dtype, self.owner.training, trainable, in_grads, backward,
                                  x.device))
        for k, t in enumerate(inputs):
            plan.set_input(f"in{k}", t)
        region, c = plan.g.outputs[self.key]
        buf = torch.empty((n, region.H, region.W, region.buf.C), dtype=torch.float32, device=x.device)
        plan.set_output(self.key, buf)
        plan.run_forward()
        if self.owner.training:  # one increment per BatchNorm call, as nn.BatchNorm2d.train()
            for op in plan.g.ops:
                if isinstance(op, E.BNOp) and op.m.num_batches_tracked is not None:
                    op.m.num_batches_tracked.add_(1)
        self.last_plan = plan
        return plan, (buf.permute(0, 3, 1, 2)[:, :c],)

    def run_backward(self, plan, inputs, grads, needs):
        (go,) = grads
        if any(p.requires_grad for p in self.params):
            plan.set_param_grads(self.owner.grad_views(self.params))
        plan.set_output_grad(self.key, go.float())
        outs = []
        for k, t in enumerate(inputs):
            if f"in{k}" in plan.ext_grad:
                gx = torch.empty(t.shape, dtype=torch.float32, device=t.device)
                plan.set_input_grad(f"in{k}", gx)
                outs.append(gx)
            else:
                outs.append(None)
        plan.run_backward()
        return outs


class _FCRunner:
    """mu_fc and logvar_fc (Linear(1024, 1024)) over the flattened code as one plan: two 1x1
    convs reading the same (B, 1, 1, 1024) buffer."""

    def __init__(self, owner, mu_fc, logvar_fc):
        self.owner = owner
        self.layers = (("mu", E.LinearAsConv(mu_fc)), ("logvar", E.LinearAsConv(logvar_fc)))
        self.params = list(mu_fc.parameters()) + list(logvar_fc.parameters())
        self.pool = PlanPool(self._build)

    def _build(self, pkey):
        n, dtype, trainable, in_grad, backward, dev = pkey
        g = E.Graph(dtype)
        fin = g.buffer("vae_code", 1, 1, 1024)
        g.input_nchw(E.R(fin), "in0", ext_c=1024, requires_grad=in_grad)
        for key, ad in self.layers:
            o = g.buffer(key, 1, 1, 1024, dtype=torch.float32, external=True)
            g.conv(E.R(fin), ad, E.R(o), trainable=trainable, name=key + "_fc")
            g.output(key, E.R(o), 1024)
        return g.compile(n, dev, backward=backward)

    def run_forward(self, inputs, train):
        (x,) = inputs  # (B, 1024, 1, 1): view(-1, 1024) of the NCHW code
        n = x.shape[0]
        needs = getattr(self, "_in_needs", (False,))
        trainable = bool(train) and any(p.requires_grad for p in self.params)
        in_grad = bool(train) and bool(needs[0])
        plan = self.pool.acquire((n, self.owner.dtype, trainable, in_grad, trainable or in_grad, x.device))
        plan.set_input("in0", x)
        outs = []
        for key, _ in self.layers:
            buf = torch.empty((n, 1, 1, 1024), dtype=torch.float32, device=x.device)
            plan.set_output(key, buf)
            outs.append(buf.view(n, 1024))
        plan.run_forward()
        return plan, tuple(outs)

    def run_backward(self, plan, inputs, grads, needs):
        (x,) = inputs
        n = x.shape[0]
        if any(p.requires_grad for p in self.params):
            plan.set_param_grads(self.owner.grad_views(self.params))
        for (key, _), gr in zip(self.layers, grads):
            gr = torch.zeros((n, 1024), device=x.device) if gr is None else gr.float()
            plan.set_output_grad(key, gr.reshape(n, 1024, 1, 1))
        gx = None
        if "in0" in plan.ext_grad:
            gx = torch.empty(x.shape, dtype=torch.float32, device=x.device)
            plan.set_input_grad("in0", gx)
        plan.run_backward()
        return [gx]


class _ReparamFn(torch.autograd.Function):
    """z = eps * exp(0.5 * logvar) + mu (nets/HRNet.py:960-964) on the HIP kernel."""

    @staticmethod
    def forward(ctx, mu, logvar, eps):
        mu, logvar, eps = mu.contiguous(), logvar.contiguous(), eps.float().contiguous()
        z = torch.empty_like(mu)
        L.check(L.load().dvie_reparam_fwd(mu.data_ptr(), logvar.data_ptr(), eps.data_ptr(), z.data_ptr(), mu.numel(),
                                          L.stream_ptr(mu.device)), "reparam")
        ctx.save_for_backward(logvar, eps)
        return z

    @staticmethod
    def backward(ctx, gz):
        logvar, eps = ctx.saved_tensors
        gz = gz.float().contiguous()
        gmu, glv = torch.empty_like(logvar), torch.empty_like(logvar)
        L.check(L.load().dvie_reparam_bwd(logvar.data_ptr(), eps.data_ptr(), gz.data_ptr(), gmu.data_ptr(),
                                          glv.data_ptr(), logvar.numel(), 0, L.stream_ptr(logvar.device)),
                "reparam backward")
        return gmu, glv, None


class VAEHRNet(HRNet):
    """Reference nets/HRNet.py:702-1061.  forward(input, gt_x, gt_seg) -> (rgb, seg, mu,
    logvar) as the reference; forward_vae(x, seg, gt_x, gt_seg, eps=None) for InterGANNet."""

    _stem_extra = 32
    post_sync = True  # data parallel: all-reduce after the whole backward (runners/comm.GradSync)

    def __init__(self, args):
        nn.Module.__init__(self)
        self._setup(args)
        if self.n_frames != 2:
            raise NotImplementedError("VAEHRNet: the reference's 23*3-channel encoder input fixes two input frames")
        self.vae_channel = 32
        self.vae_encoder = nn.Sequential(
            Conv2d(23 * 3, 32, 3, 1, 1), nn.LeakyReLU(0.2, inplace=True),
            *_cbl(32, 32), *_cbl(32, 32, 2), *_cbl(32, 32), *_cbl(32, 64, 2), *_cbl(64, 64),
            *_cbl(64, 128, 2), *_cbl(128, 128), *_cbl(128, 128, 2), *_cbl(128, 64), *_cbl(64, 32),
            Conv2d(32, 16, 3, 1, 1))
        self.mu_fc = nn.Linear(1024, 1024)
        self.logvar_fc = nn.Linear(1024, 1024)
        self.vae_decoder = nn.Sequential(
            *_tbl(16, 32), *_cbl(32, 32), *_tbl(32, 32), *_cbl(32, 32), *_tbl(32, 32), *_cbl(32, 32),
            *_tbl(32, 32), Conv2d(32, 32, 3, 1, 1))
        self._build_trunk()
        self._finish()
        vae_ids = {id(p) for m in (self.vae_encoder, self.mu_fc, self.logvar_fc, self.vae_decoder)
                   for p in m.parameters()}
        self._trunk = [p for p in self._flat_params if id(p) not in vae_ids]
        self._enc = _SeqRunner(self, self.vae_encoder, "vae_encoder", [6, 40, 3, 20], "vae_code")
        self._fc = _FCRunner(self, self.mu_fc, self.logvar_fc)
        self._dec = _SeqRunner(self, self.vae_decoder, "vae_decoder", [16], "vae_feature")

    def _trunk_params(self):
        return self._trunk

    def _on_moved(self):
        super()._on_moved()
        for r in (self._enc, self._fc, self._dec):
            r.pool.clear()

    def forward_vae(self, x, seg, gt_x=None, gt_seg=None, eps=None):
        x, seg = x.float(), seg.float()
        n = x.shape[0]
        mu = logvar = None
        if self.training:
            code = PlanFunction.apply(self._enc, 4, x, seg, gt_x.float(), gt_seg.float(), *self._enc.params)
            mu, logvar = PlanFunction.apply(self._fc, 1, code.reshape(n, 1024, 1, 1), *self._fc.params)
            if eps is None:
                eps = torch.randn_like(mu)  # std.new(std.size()).normal_()
            self.last_eps = eps  # the step's noise (test support: the oracle replays it)
            z = _ReparamFn.apply(mu, logvar, eps.to(mu.device))
        else:  # torch.zeros(bs, 1024).normal_()
            z = (torch.randn(n, 1024, device=x.device) if eps is None else eps.to(x.device)).float()
        vae = PlanFunction.apply(self._dec, 1, z.reshape(n, 16, 8, 8), *self._dec.params)
        rgb, seg_out = PlanFunction.apply(self, 3, x, seg, vae, *self._trunk)
        return rgb, seg_out, mu, logvar

    def forward(self, input, gt_x=None, gt_seg=None):
        F = self.n_frames
        x, seg = input[:, :3 * F], input[:, 3 * F:3 * F + 20 * F]
        return self.forward_vae(x, seg, gt_x, gt_seg)
