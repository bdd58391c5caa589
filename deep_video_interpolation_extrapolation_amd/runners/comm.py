"""Data-parallel gradient synchronisation over RCCL (torch.distributed 'nccl' on ROCm).

Replaces DistributedDataParallel (runners/InterTrainer.py:63-64) for plan-executed models:
parameters live in one flat fp32 buffer laid out in backward-completion order, so the
gradient all-reduce is a handful of large contiguous buckets launched from inside the
backward pass as soon as each bucket's weight reductions are enqueued (RCCL runs on its
own stream, overlapping the remaining backward kernels).  The loss-value sync of the
reference (`sync`, l.859-864: one all_reduce per scalar) is one coalesced all_reduce.

Gradient scaling follows the reference exactly: each rank back-propagates loss_all / W
(the in-place div_ of `sync` is recorded by autograd) and DDP averages, so the applied
gradient is (1/W) * mean_r grad(L_r); here: SUM all-reduce, then x 1/W.
"""
import os

import torch
import torch.distributed as dist

from .. import _lib as L


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class GradSync:
    """`self.model = GradSync(model)` keeps `self.model.module` like DDP does."""

    def __init__(self, module, bucket_mb=None):
        self.module = module
        self.W = world()
        self.bucket_bytes = int(float(bucket_mb or os.environ.get("DVIE_BUCKET_MB", 16)) * 2 ** 20)
        self.flat_owners = [m for m in module.modules() if hasattr(m, "_flat")]
        # owners that launch their buckets from inside their backward (HRNet); the others
        # (discriminators, a few MB, gradients accumulated over two plan backwards) get one
        # all-reduce of their flat gradient after the backward
        # (VAEHRNet: parameters of several chained plans share one flat buffer, so it syncs
        # after its whole backward)
        self.hooked = [m for m in self.flat_owners if hasattr(m, "_buckets") and not getattr(m, "post_sync", False)]
        self.post = [m for m in self.flat_owners if m not in self.hooked]
        self.works = []
        self.overlap = True
        if self.W > 1:
            for m in self.flat_owners:  # DDP's initial parameter broadcast
                dist.broadcast(m._flat, 0)
            for m in self.hooked:
                m.grad_hook = (self.bucket_bytes, self._make_hook(m))

    def set_overlap(self, flag):
        """In-backward bucket all-reduces on (default) or off.  Off when a step runs the
        same model's backward more than once (ExtraTrainer's num_pred_step > 1 rollout):
        a later backward accumulates into the flat gradient (beta = 1), so reducing after
        the first one would race its in-flight buckets and count the earlier gradient W
        times; the flat gradient is then reduced once in finish()."""
        flag = bool(flag)
        if flag == self.overlap:
            return
        self.overlap = flag
        if self.W > 1:
            for m in self.hooked:
                m.grad_hook = (self.bucket_bytes, self._make_hook(m)) if flag else None

    # hipGraph capture of the backward (runners/graph.py): while capturing, a callable
    # fn(owner, lo, hi) the bucket hooks hand each finished bucket to (it closes the captured
    # graph segment there) instead of launching the all-reduce
    capture_cut = None

    def _make_hook(self, owner):
        def hook(lo, hi):
            if hi <= lo:
                return
            if self.capture_cut is not None:
                self.capture_cut(owner, lo, hi)
                return
            self.works.append(dist.all_reduce(owner._flat_grad[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
        return hook

    def reduce_bucket(self, owner, lo, hi):
        """A replayed graph segment's finished bucket: its all-reduce on the communication
        stream, ordered after the work enqueued so far on the current stream (the segment),
        so it runs while the next segments replay."""
        if self.W == 1:
            return
        g = owner._flat_grad
        if not g.is_cuda:  # host tensors (the CPU gloo tests)
            self.works.append(dist.all_reduce(g[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
            return
        comm = self.comm_stream()
        comm.wait_stream(torch.cuda.current_stream(g.device))
        with torch.cuda.stream(comm):
            self.works.append(dist.all_reduce(g[lo:hi], op=dist.ReduceOp.SUM, async_op=True))

    def reduce_rest(self, bucketed):
        """After the replayed backward: the all-reduces not issued per bucket (every flat
        owner if no buckets were, else the post-backward owners), then wait for all."""
        if self.W == 1:
            return
        for m in (self.post if bucketed else self.flat_owners):
            if m._flat_grad is not None and any(p.grad is not None for p in m.parameters()):
                self.works.append(dist.all_reduce(m._flat_grad, op=dist.ReduceOp.SUM, async_op=True))
        self.wait()

    _comm = None

    def comm_stream(self):
        if self._comm is None:
            self._comm = torch.cuda.Stream(self.flat_owners[0]._flat.device)
        return self._comm

    def __call__(self, *a, **k):
        return self.module(*a, **k)

    def __getattr__(self, name):
        return getattr(self.__dict__["module"], name)

    def wait(self):
        """Join the bucket all-reduces (stream-ordered on the GPU)."""
        for w in self.works:
            w.wait()
        self.works = []

    def finish(self):
        """Wait for the bucket all-reduces and apply the 1/W factor (HIP kernel)."""
        if self.W == 1:
            return
        self.reduce()
        self.scale()

    def reduce(self):
        """The collectives of finish(): the post-backward all-reduces, then wait for all."""
        if self.W == 1:
            return
        for m in (self.post if self.overlap else self.flat_owners):
            if m._flat_grad is not None and any(p.grad is not None for p in m.parameters()):
                self.works.append(dist.all_reduce(m._flat_grad, op=dist.ReduceOp.SUM, async_op=True))
        self.wait()

    def scale(self):
        """The 1/W factor of finish() (device work only: graph-capturable)."""
        if self.W == 1:
            return
        lib = L.load()
        for m in self.flat_owners:
            g = m._flat_grad
            if g is not None:
                L.require_gpu(g)
                L.check(lib.dvie_scale(g.data_ptr(), g.numel(), 1.0 / self.W, L.stream_ptr(g.device)), "grad scale")

    def train(self, mode=True):
        self.module.train(mode)
        return self

    def eval(self):
        return self.train(False)


def sync_losses(loss_dict, W):
    """Mean over ranks of every logged scalar, as one all_reduce (values only)."""
    if W == 1:
        return loss_dict
    keys = list(loss_dict.keys())
    flat = torch.stack([loss_dict[k].detach().float().reshape(()) for k in keys])
    dist.all_reduce(flat)
    flat /= W
    for i, k in enumerate(keys):
        loss_dict[k] = flat[i]
    return loss_dict
