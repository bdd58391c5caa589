"""hipGraph-captured training step (BASELINE config 5: "hipGraph-captured step").

The engine already runs a whole network pass as one host call per plan, but a step is
still ~600-1,000 kernel launches (HRNet + VGG forward and backward, losses, optimizer).
`GraphedStep` records one complete trainer step -- forward, losses, backward, 1/W
scaling, optimizer updates -- into a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm)
and replays it: one launch per step, no Python or driver work per kernel.

* Inputs are static: each call copies the batch into the captured input tensors (or the
  caller passes those tensors, `GraphedStep.inputs`, to skip the copy).
* Optimizers switch to their capturable form (device-resident step counts,
  optim._FusedOptimizer.set_capturable), so bias corrections advance on replay.
* W == 1: the whole step is one graph.  W > 1: collectives are not captured.  The
  forward + backward is captured as a chain of graph segments that end where the eager
  backward would launch a gradient bucket's all-reduce (runners/comm.py: the bucket hook
  closes the segment and opens the next one on the capture stream); on replay, after each
  segment its bucket's RCCL all-reduce is issued on a communication stream ordered after
  that segment, so it overlaps the following segments as the eager in-backward buckets do;
  then the remaining all-reduces and the wait (GradSync.reduce_rest), then graph 2 = 1/W
  scale + optimizer steps, then the eager loss-value all-reduce.  (A step whose backward
  accumulates twice -- ExtraTrainer's rollout -- has no buckets: one segment, then the
  flat gradients' all-reduces.)
* The warm-up steps before capture (on a side stream, as stream capture requires) are real
  training steps; capture itself executes nothing.
"""
from collections import OrderedDict

import torch

from . import comm


class GraphedStep:
    def __init__(self, trainer, example, warmup=2):
        assert warmup >= 1, "one eager step must run before capture (it builds the plans and moves step counts)"
        self.tr = trainer
        dev = trainer.device
        self.inputs = {k: v.to(dev).clone() for k, v in example.items()}
        self.split = trainer.W > 1
        self.segments = []
        opts = trainer._opts()
        for o in opts:
            o.set_capturable(True)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                trainer.step(self.inputs)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        g0 = trainer.global_step
        if not self.split:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = trainer.step(self.inputs)
            self.graphs = (self.graph,)
        else:
            pool = torch.cuda.graph_pool_handle()
            self.segments = []  # [(graph, bucket (owner, lo, hi) finished at its end, or None)]
            self._tick = torch.zeros(1, device=dev)
            cur = [torch.cuda.CUDAGraph()]

            def cut(owner, lo, hi):  # on the backward's thread and capture stream
                cur[0].capture_end()
                self.segments.append((cur[0], (owner, lo, hi)))
                cur[0] = torch.cuda.CUDAGraph()
                cur[0].capture_begin(pool=pool, capture_error_mode="relaxed")

            torch.cuda.synchronize(dev)
            # relaxed capture: the segments end and begin on autograd's backward thread
            with torch.cuda.stream(side):
                cur[0].capture_begin(pool=pool, capture_error_mode="relaxed")
                trainer.model.capture_cut = cut
                try:
                    self.out = trainer.forward_backward(self.inputs)
                    self._tick.add_(1)  # the last segment is never empty
                finally:
                    trainer.model.capture_cut = None
                    cur[0].capture_end()
                self.segments.append((cur[0], None))
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph2, pool=pool):
                trainer.apply_gradients(reduce=False)
            self.graph = self.segments[0][0]
            self.graphs = tuple(g for g, _ in self.segments) + (self.graph2,)
        trainer.global_step = g0  # capture ran no step

    def close(self):
        """Give the trainer back its eager form: optimizers leave capturable mode (step counts
        return to the host, as checkpoints store them).  The captured graphs are released."""
        tr = self.tr
        for o in tr._opts():
            o.set_capturable(False)
        self.graph = self.graph2 = None
        self.segments = []
        self.graphs = ()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __call__(self, data=None):
        return self.step(data)

    def step(self, data=None):
        """One training step: copy `data` (if given and not the static inputs) into the
        captured inputs and replay.  Returns the loss dict (tensors owned by the graph,
        overwritten by the next replay)."""
        if data is not None and data is not self.inputs:
            for k, v in data.items():
                t = self.inputs[k]
                if v.data_ptr() != t.data_ptr():
                    t.copy_(v, non_blocking=True)
        tr = self.tr
        if not self.split:
            self.graph.replay()
            tr.global_step += 1
            return self.out
        for g, bucket in self.segments:
            g.replay()
            if bucket is not None:
                tr.model.reduce_bucket(*bucket)
        tr.model.reduce_rest(len(self.segments) > 1)
        self.graph2.replay()
        tr.global_step += 1
        return comm.sync_losses(OrderedDict((k, v.clone()) for k, v in self.out.items()), tr.W)
