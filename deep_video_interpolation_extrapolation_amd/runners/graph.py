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
* W == 1: the whole step is one graph.  W > 1: collectives are not captured; graph 1 =
  forward + backward, in which every gradient bucket the eager backward would all-reduce
  in flight (runners/comm.py) ends with an external event-record node instead; on replay
  each bucket's RCCL all-reduce is issued on a communication stream waiting for its event
  (GradSync.reduce_replayed), so it overlaps the rest of the replayed backward as the eager
  step's does; then graph 2 = 1/W scale + optimizer steps, then the eager loss-value
  all-reduce.  (A step whose backward accumulates twice -- ExtraTrainer's rollout --
  records no bucket events: its flat gradients are reduced after graph 1.)
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
        self.events = []
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
            self.graph = torch.cuda.CUDAGraph()
            trainer.model.capture_events = []  # bucket hooks record events, launch nothing
            try:
                with torch.cuda.graph(self.graph):
                    self.out = trainer.forward_backward(self.inputs)
            finally:
                self.events = trainer.model.capture_events
                trainer.model.capture_events = None
            self.graph2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph2, pool=self.graph.pool()):
                trainer.apply_gradients(reduce=False)
            self.graphs = (self.graph, self.graph2)
        trainer.global_step = g0  # capture ran no step

    def close(self):
        """Give the trainer back its eager form: optimizers leave capturable mode (step counts
        return to the host, as checkpoints store them).  The captured graphs are released."""
        tr = self.tr
        for o in tr._opts():
            o.set_capturable(False)
        self.graph = self.graph2 = None
        self.events = []
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
        self.graph.replay()
        if not self.split:
            tr.global_step += 1
            return self.out
        tr.model.reduce_replayed(self.events)
        self.graph2.replay()
        tr.global_step += 1
        return comm.sync_losses(OrderedDict((k, v.clone()) for k, v in self.out.items()), tr.W)
