"""GPU: hipGraph-captured training steps (runners/graph.py) replay the eager step.

For each trainer, trainer A runs N eager steps and trainer B (same seed) runs 2 eager
warm-up steps + capture + N-2 replays on the same batch: the loss dicts of every step and
the final parameters must agree (the captured Adamax / Adam compute their bias correction
on the device from a device step count: ~1e-7 relative differences from the host's double
arithmetic on the float32 beta are the only expected deviation)."""
import numpy as np
import pytest
import torch

import inputs
from oracle import step as OS

pytestmark = pytest.mark.gpu


def _args(runner="INTER", **kw):
    from deep_video_interpolation_extrapolation_amd.options import default_args
    a = default_args(runner, syn_type="inter" if runner == "INTER" else "extra")
    a.__dict__.update(train_coarse=True, batch_size=2, input_h=64, input_w=128, precision="fp32", synthetic=2,
                      num_workers=0, split="train")
    a.__dict__.update(kw)
    return a


def _make(kind, **kw):
    if kind == "extra":
        from deep_video_interpolation_extrapolation_amd.runners.ExtraTrainer import ExtraTrainer as T
        a = _args("EXTRA", **kw)
    elif kind == "gan":
        from deep_video_interpolation_extrapolation_amd.runners.InterGANTrainer import InterGANTrainer as T
        a = _args(model="InterGANNet", gan=True, frame_disc=True, video_disc=True, train_frame_disc=True,
                  train_video_disc=True, seg_disc=True, input_h=128, input_w=128, **kw)
    else:
        from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer as T
        a = _args(**kw)
    torch.manual_seed(1024)
    return T(a)


def _flats(tr):
    return [m._flat.detach().clone() for m in tr.model.flat_owners]


CASES = [("inter", {}), ("inter", dict(model="InterStage3Net", refine=True, refine_model="SRNRefine", stage3=True, train_refine=True,
                                       train_stage3=True, n_scales=2)),
         ("extra", dict(num_pred_step=2)), ("gan", {})]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind,kw", CASES, ids=["inter", "inter_stage3", "extra_rollout", "intergan"])
def test_graphed_step_replays_eager(dev, kind, kw):
    from deep_video_interpolation_extrapolation_amd.runners.graph import GraphedStep
    N = 5
    frames = 4 if kind == "extra" else 3
    H, W = (128, 128) if kind == "gan" else (64, 128)
    from deep_video_interpolation_extrapolation_amd.data import SyntheticClips
    ds = SyntheticClips(2, H, W, frames)
    items = [ds[i] for i in range(2)]
    data = {k: torch.stack([it[k] for it in items]).to(dev) for k in items[0]}
    a = _make(kind, **kw)
    eager = [{k: float(v) for k, v in a.step(data).items()} for _ in range(N)]
    b = _make(kind, **kw)
    gs = GraphedStep(b, data, warmup=2)
    graphed = []
    for _ in range(N - 2):
        out = gs.step(data)
        graphed.append({k: float(v) for k, v in out.items()})
    torch.cuda.synchronize()
    assert b.global_step == a.global_step
    for e, g in zip(eager[2:], graphed):
        assert list(e) == list(g)
        np.testing.assert_allclose([g[k] for k in e], [e[k] for k in e], rtol=2e-5, atol=1e-7)
    for fa, fb in zip(_flats(a), _flats(b)):
        assert float((fa - fb).abs().max()) <= 1e-5 * max(1.0, float(fa.abs().max())), float((fa - fb).abs().max())
