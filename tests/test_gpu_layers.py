"""GPU: layer-local parity of every op the timed bf16 training step runs (BASELINE config 2:
InterNet 256x512, bf16, batch 8 -- the step bench.py times), against a float64 torch
evaluation of that op on its own stored operands.

The step runs once with engine.OP_HOOK = plan_ref.Checker: each descriptor of the HRNet and
VGG19 plans (weight pack, convolutions forward and data gradient in every stride phase, weight
gradients and their slab reductions, bias column sums, the fused rgb-head and seg-encoder
backwards, the pointwise fuse / upsample-adjoint / pool / copy / pack ops, the feature-L1 loss
ops) is evaluated by the interpreter of tests/plan_ref.py from the bf16 activations, packed
bf16 weights and fp32 slabs the kernel itself reads, then launched through the C ABI with the
library's launch trace on (dvie_trace_kernels), and compared:
* a stored bf16 activation / gradient: relative L2 <= 4e-3 (bf16 output rounding);
* fp32 results (the fp32 head outputs, parameter gradients after the slab reduction, loss
  values, the NCHW input gradient): <= 1e-4;
* weight-gradient / bias partial slabs, summed over the slabs: <= 1e-4;
* packed weights: bit-exact;
* and no byte of an output buffer outside the op's region changed.
The interpreter itself is pinned to the fp64 oracle on the CPU (tests/test_plan_ref_cpu.py).
One line per op is printed: list, index, layer, kernel(s), error.
Reference: nets/HRNet.py:339-601, nets/vgg.py:11-54, losses.py:157-180 of the reference."""
import os
import sys

import pytest
import torch

from plan_ref import Checker, Memory, track

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trainer(dev, batch, H, W):
    sys.path.insert(0, ROOT)
    from bench import make_batch
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer

    class _Log:
        def info(self, msg):
            pass

    args = default_args("INTER", syn_type="inter", interval=5, mode="xs2xs", vid_length=1, train_coarse=True,
                        batch_size=batch, input_h=H, input_w=W, precision="bf16", synthetic=batch, num_workers=0,
                        split="train", rank=0, gpus=1)
    args.logger = _Log()
    torch.manual_seed(args.seed)
    return InterTrainer(args), make_batch(batch, H, W, dev, 0)


KIND = {1: "conv", 2: "wgrad", 3: "wreduce", 4: "colsum", 5: "ew", 6: "loss", 7: "pack", 13: "head3_bwd",
        14: "segenc_fwd", 15: "segenc_bwd", 16: "wreduce*"}


@pytest.mark.parametrize("batch,H,W", [(8, 256, 512), (2, 48, 80)], ids=["c2_8x256x512", "ragged_2x48x80"])
def test_every_op_of_the_bf16_step_matches_its_reference(dev, monkeypatch, batch, H, W):
    from deep_video_interpolation_extrapolation_amd import engine as E
    monkeypatch.setenv("DVIE_PRECISION", "bf16")
    torch.backends.cuda.matmul.allow_tf32 = False
    trainer, data = _trainer(dev, batch, H, W)
    mem = Memory(dev)
    track(mem, monkeypatch.setattr)
    for t in data.values():
        mem.add(t)
    chk = Checker(mem)
    monkeypatch.setattr(E, "OP_HOOK", chk)
    trainer.step(data)
    torch.cuda.synchronize()
    monkeypatch.setattr(E, "OP_HOOK", None)
    per_kernel = {}
    for i, r in enumerate(chk.records):
        ks = r["kernels"].split(";") if r["kernels"] else ["-"]
        short = ",".join(k.split("(")[0] for k in ks)
        err = "-" if r["err"] is None else f"{r['err']:.2e}"
        print(f"op {i:4d} {KIND.get(r['kind'], r['kind']):10s} {r['name'][:38]:38s} {err:>8s} {short[:120]}")
        for k in ks:
            name = k.split("(")[0]
            w = per_kernel.setdefault(name, [0, 0.0])
            w[0] += 1
            if r["err"] is not None and r["bar"]:
                w[1] = max(w[1], r["err"] / r["bar"])
    print(f"{len(chk.records)} ops; per kernel (ops, worst error / bar):")
    for k, (n, w) in sorted(per_kernel.items(), key=lambda kv: -kv[1][0]):
        print(f"  {n:4d} {w:6.3f}  {k}")
    assert not chk.failures, chk.failures[:10]
    assert all(r["checked"] for r in chk.records)
    kinds = {r["kind"] for r in chk.records}
    assert {1, 2, 5, 6, 7, 13, 14, 15} <= kinds and (3 in kinds or 16 in kinds), kinds
    if (batch, H, W) == (8, 256, 512):
        names = " ".join(per_kernel)
        for k in ("conv_h8_kernel", "conv_strip_kernel", "conv1x1_kernel", "conv1x1_ring_kernel", "conv_s2_kernel",
                  "wgrad_halo_kernel", "wgrad_wide_kernel", "head3_bwd_kernel", "segenc_fwd_kernel", "segenc_bwd_kernel", "pack_kernel",
                  "wreduce_multi_kernel", "ew_fuse2_kernel", "ew_fuser_kernel", "ew_upt22_kernel", "ew_nchw_kernel"):
            assert k in names, (k, sorted(per_kernel))
