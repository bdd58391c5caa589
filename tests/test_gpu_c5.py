"""GPU: BASELINE config 5 as one workload -- the two-stage extrapolation net
(ExtraStage3Net: HRNet coarse + SRNRefine + MSResAttnRefine, build-defined because the
reference has no runnable two-stage extrapolation model) trained by
ExtraTrainer --refine --stage3, as a hipGraph-captured step at 1024x2048.

* fp32 step at 64x128 (n_sc 2, stage3_prop) vs oracle.step.extra_refine_step: loss dict in
  the reference key order within 1e-4, gradients of all three nets, post-Adamax weights;
* the captured bf16 step at 1024x2048 (batch 1, n_sc 3, stage3_prop, all three nets
  trained: the bench's `--workload c5`) replays the eager step: trainer A runs 4 eager
  steps, trainer B 2 eager warm-up steps + capture + 2 replays, loss dicts and final
  parameters agree;
* bf16 output quality of the two-stage forward at 1024x2048 against the fp32 path
  (coarse, last refine and last stage-3 image): PSNR and relative L2 gated.
"""
import gc
import math

import numpy as np
import pytest
import torch

import inputs
from oracle import hrnet as OH
from oracle import losses as OL
from oracle import refine as OR
from oracle import step as OS

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(1e-30, float(b.norm())))


def _args(**kw):
    from deep_video_interpolation_extrapolation_amd.options import default_args
    a = default_args("EXTRA", syn_type="extra", model="ExtraStage3Net", refine=True, refine_model="SRNRefine",
                     stage3=True, train_coarse=True, train_refine=True, train_stage3=True, num_workers=0,
                     split="train")
    a.__dict__.update(kw)
    return a


def _trainer(**kw):
    from deep_video_interpolation_extrapolation_amd.runners.ExtraTrainer import ExtraTrainer
    torch.manual_seed(1024)
    return ExtraTrainer(_args(**kw))


@pytest.mark.timeout(300)
def test_extra_stage3_step_matches_oracle(dev, monkeypatch):
    """Loss dict 1e-4; every gradient tensor of the three nets within 1e-4 relative L2 of the
    fp64 oracle evaluated on this step's branches (coarse HRNet LeakyReLUs, refine and stage-3
    activation lists, the ReLUs of each VGG-loss call); post-Adamax weights."""
    from deep_video_interpolation_extrapolation_amd.nets.vgg import my_vgg
    tr = _trainer(n_scales=2, stage3_prop=True, batch_size=2, input_h=64, input_w=128, synthetic=2,
                  precision="fp32")
    data = OS.synthetic_batch(2, 64, 128)
    monkeypatch.setattr(my_vgg, "sign_log", [])
    ld = tr.step(data)
    vmasks = my_vgg.sign_log
    Pc = OH.init_params(1024)
    Pr = OR.init_params(None, OR.srn_specs())
    Ps = OR.init_params(None, OR.attn_specs())
    ref, _, new = OS.extra_refine_step(Pc, Pr, OL.synthetic_vgg19_state(), data, 2, Ps=Ps, prop=True)
    assert list(ld.keys()) == list(ref.keys()), (list(ld.keys()), list(ref.keys()))
    np.testing.assert_allclose([float(ld[k]) for k in ref], [ref[k] for k in ref], rtol=1e-4)
    m = tr.model.module
    _, g64, _ = OS.extra_refine_step(Pc, Pr, OL.synthetic_vgg19_state(), data, 2, Ps=Ps, prop=True,
                                     masks=m.coarse_model.last_plan.activation_signs(),
                                     rmasks=m.refine_model.last_plan.activation_list(),
                                     smasks=m.stage3_model.last_plan.activation_list(), vmasks=vmasks,
                                     dtype=torch.float64)
    for part, mod in (("coarse", m.coarse_model), ("refine", m.refine_model), ("stage3", m.stage3_model)):
        named = dict(mod.named_parameters())
        errs = {k: rel_l2(named[k].grad, g) for k, g in g64[part].items()}
        worst = max(errs, key=errs.get)
        print(f"C5-net step {part}: gradients vs fp64 oracle on the same branches: relative L2 median "
              f"{np.median(list(errs.values())):.2e}, worst {errs[worst]:.2e} ({worst})")
        assert errs[worst] <= 1e-4, (part, worst, errs[worst])
        moved = sum(int(((named[k].detach().cpu() - w).abs() > 1e-4).sum()) for k, w in new[part].items())
        total = sum(w.numel() for w in new[part].values())
        assert moved <= 1e-3 * total, (part, moved, total)


C5 = dict(n_scales=3, stage3_prop=True, batch_size=1, input_h=1024, input_w=2048, synthetic=1, precision="bf16")


def _c5_batch(dev):
    from deep_video_interpolation_extrapolation_amd.data import SyntheticClips
    ds = SyntheticClips(1, 1024, 2048, 3)
    it = ds[0]
    return {k: v.unsqueeze(0).to(dev) for k, v in it.items()}


@pytest.mark.timeout(900)
def test_c5_graphed_two_stage_step_replays_eager(dev):
    from deep_video_interpolation_extrapolation_amd.runners.graph import GraphedStep
    data = _c5_batch(dev)
    N = 4
    a = _trainer(**C5)
    eager = [{k: float(v) for k, v in a.step(data).items()} for _ in range(N)]
    flats_a = [m._flat.detach().float().cpu() for m in a.model.flat_owners]
    del a
    gc.collect()
    torch.cuda.empty_cache()
    b = _trainer(**C5)
    gs = GraphedStep(b, data, warmup=2)
    graphed = [{k: float(v) for k, v in gs.step().items()} for _ in range(N - 2)]
    torch.cuda.synchronize()
    assert b.global_step == N
    worst = 0.0
    for e, g in zip(eager[2:], graphed):
        assert list(e) == list(g)
        assert all(np.isfinite(v) for v in g.values()), g
        worst = max(worst, max(abs(g[k] - e[k]) / max(1e-12, abs(e[k])) for k in e))
    print(f"C5 captured vs eager: {len(eager[0])} losses per step, worst relative difference {worst:.2e}; "
          f"loss_all eager {[e['loss_all'] for e in eager]} graphed {[g['loss_all'] for g in graphed]}")
    assert worst < 2e-4, worst
    for fa, m in zip(flats_a, b.model.flat_owners):
        fb = m._flat.detach().float().cpu()
        assert float((fa - fb).abs().max()) <= 1e-5 * max(1.0, float(fa.abs().max())), float((fa - fb).abs().max())
    gs.close()
    del gs, b
    gc.collect()
    torch.cuda.empty_cache()


def _psnr_pm1(a, b):
    mse = float((((a + 1) / 2 - (b + 1) / 2) ** 2).mean())
    return 10 * math.log10(1.0 / max(mse, 1e-20))


@pytest.mark.timeout(600)
def test_c5_two_stage_bf16_quality_vs_fp32(dev):
    """Same weights, same 1024x2048 input: the bf16 two-stage forward against the fp32 one
    (the fp32 path is the oracle-parity mode, pinned at 64x128 above and in
    test_gpu_refine): PSNR >= 40 dB on the coarse, last refine and last stage-3 images
    (mapped from [-1, 1] to [0, 1]) and relative L2 < 5e-2."""
    from deep_video_interpolation_extrapolation_amd import nets
    gc.collect()
    torch.cuda.empty_cache()
    x, seg = inputs.hrnet_input(1, 1024, 2048)
    outs = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(1024)
        m = nets.ExtraStage3Net(_args(n_scales=3, stage3_prop=True, precision=prec)).to(dev).eval()
        with torch.no_grad():
            c_rgb, _, ref, re, _ = m(x.to(dev), seg=seg.to(dev))
        outs[prec] = [t.detach().float().cpu() for t in (c_rgb, ref[-1], re[-1])]
        del m, c_rgb, ref, re
        gc.collect()
        torch.cuda.empty_cache()
    res = [(_psnr_pm1(b, f), rel_l2(b, f)) for b, f in zip(outs["bf16"], outs["fp32"])]
    print("C5 bf16 vs fp32 (coarse, refine, stage3): PSNR dB / relative L2 " +
          ", ".join(f"{p:.1f} / {r:.2e}" for p, r in res))
    assert all(p >= 40.0 for p, _ in res) and all(r < 5e-2 for _, r in res), res
