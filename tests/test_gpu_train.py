"""GPU: one full InterTrainer step (HRNet plan + RGBLoss + CE + backward + Adamax) in fp32
parity mode against the reference step fixture (tests/golden/step.npz), and bf16 sanity."""
import os

import numpy as np
import pytest
import torch

import inputs

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def trainer(prec, H, W, B, **kw):
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer
    args = default_args("INTER", syn_type="inter", train_coarse=True, batch_size=B, input_h=H, input_w=W,
                        precision=prec, synthetic=B, num_workers=0, split="train", **kw)
    os.environ["DVIE_PRECISION"] = prec
    torch.manual_seed(1024)
    return InterTrainer(args)


def test_inter_step_matches_reference(dev):
    """Loss dict within 1e-4 relative; gradient sums of squares within 1e-3 (median) /
    2e-2 (worst) relative of the reference's (LeakyReLU kink flips, see test_gpu_parity),
    and every gradient tensor within 1e-4 relative L2 of the fp64 oracle evaluated on this
    step's activation branches; post-Adamax weight
    sums of squares within 1e-4 relative: Adamax's first step moves EVERY weight by
    +-lr whatever |grad| is, so gradients that are ~0 in both paths but of opposite sign
    move single weights by 2e-3 (the update rule itself is checked exactly in
    test_adamax_matches_torch)."""
    f = np.load(os.path.join(G, "step.npz"))
    tr = trainer("fp32", 32, 64, 2)
    ld = tr.step(inputs.step_batch(2, 32, 64))
    names = [str(n) for n in f["loss_names"]]
    assert list(ld.keys()) == names
    got = np.array([float(ld[k]) for k in names])
    np.testing.assert_allclose(got, f["loss_values"], rtol=1e-4)
    named = dict(tr.model.module.coarse_model.named_parameters())
    pn = [str(n) for n in f["param_names"]]
    g2 = np.array([float((named[n].grad.double() ** 2).sum()) for n in pn])
    rel = np.abs(g2 - f["grad_stats"][:, 1]) / f["grad_stats"][:, 1]  # relative sum-of-squares difference
    assert float(np.median(rel)) < 1e-3 and float(rel.max()) < 2e-2, (float(np.median(rel)), float(rel.max()))
    post = np.array([float((named[n].detach().double() ** 2).sum()) for n in pn])
    np.testing.assert_allclose(post, f["post_checksums"][:, 1], rtol=1e-4)
    # the same step's gradients against the fp64 oracle (pinned to this fixture by
    # test_oracle_golden) evaluated on the HIP step's own activation branches
    from oracle import hrnet as OH
    from oracle import losses as OL
    from oracle import step as OS
    masks = tr.model.module.coarse_model.last_plan.activation_signs()
    vmasks = tr.RGBLoss.vgg_loss.vgg_net.last_plan.activation_signs()
    _, g64, _, _, _ = OS.inter_step(OH.init_params(1024), OL.synthetic_vgg19_state(), inputs.step_batch(2, 32, 64),
                                    masks=masks, vmasks=vmasks, dtype=torch.float64)
    errs = {k: float((named[k].grad.double().cpu() - g).norm() / g.norm()) for k, g in g64.items()}
    worst = max(errs, key=errs.get)
    print(f"step gradients vs fp64 oracle on the same branches: median {np.median(list(errs.values())):.2e}, "
          f"worst {errs[worst]:.2e} ({worst})")
    assert errs[worst] <= 1e-4, (worst, errs[worst])


def _tape_step(prec, mode, data, monkeypatch, **kw):
    monkeypatch.setenv("DVIE_LOSS_TAPE", mode)
    tr = trainer(prec, 64, 128, 2, **kw)
    ld = tr.forward_backward(data)
    named = dict(tr.model.module.coarse_model.named_parameters())
    return ({k: float(v) for k, v in ld.items()},
            {k: p.grad.detach().double().cpu() for k, p in named.items() if p.grad is not None})


def _rel(a, b):
    return {k: float((a[k] - b[k]).norm() / max(1e-30, float(b[k].norm()))) for k in b}


def test_loss_tape_matches_autograd_losses(dev, monkeypatch):
    """losses.LossTape (the kernels write the weighted loss values and the loss gradients,
    one dvie_sum_f32 for loss_all, autograd driven from the predictions) against the
    per-term autograd form of the reference loss code (DVIE_LOSS_TAPE=0) on one step.
    fp32: same keys in the same order, values within 1e-6 relative, every HRNet gradient
    within 1e-5 relative L2 (the forms add the four image-loss gradients in different
    orders).  bf16: the tape scales the VGG plan's backward seeds by the loss weight where
    the autograd form scales its result, so the bf16 VGG backward rounds differently
    (r03o: median 3e-3 apart); gated as equally good -- each form's gradients against the
    fp32 ones, the tape's median error within 1.25x the autograd form's (+1e-4)."""
    data = inputs.step_batch(2, 64, 128)
    la, ga = _tape_step("fp32", "0", data, monkeypatch)
    lt, gt = _tape_step("fp32", "1", data, monkeypatch)
    assert list(la) == list(lt), (list(la), list(lt))
    for k in la:
        assert abs(la[k] - lt[k]) <= 1e-6 * max(1.0, abs(la[k])), (k, la[k], lt[k])
    assert set(ga) == set(gt) and ga
    errs = _rel(gt, ga)
    worst = max(errs, key=errs.get)
    print(f"fp32: loss tape vs autograd losses: {len(la)} values, gradient relative L2 median "
          f"{np.median(list(errs.values())):.2e} worst {errs[worst]:.2e} ({worst})")
    assert errs[worst] <= 1e-5, (worst, errs[worst])
    _, gab = _tape_step("bf16", "0", data, monkeypatch)
    ltb, gtb = _tape_step("bf16", "1", data, monkeypatch)
    assert list(ltb) == list(la)
    ea, et = np.median(list(_rel(gab, ga).values())), np.median(list(_rel(gtb, ga).values()))
    print(f"bf16 gradients vs fp32: autograd form median {ea:.2e}, tape {et:.2e}")
    assert et <= 1.25 * ea + 1e-4, (et, ea)


@pytest.mark.parametrize("zero", ["ssim_weight", "vgg_weight"])
def test_loss_tape_zero_weight_term(dev, monkeypatch, zero):
    """A loss term of weight 0 (--ssim_w 0 / --vgg_w 0) reports 0 in the loss dict and adds
    nothing to loss_all, in the tape as in the autograd form and the reference
    (losses.py:223-241 multiplies each term by its weight); gradients as the autograd form."""
    data = inputs.step_batch(2, 64, 128)
    la, ga = _tape_step("fp32", "0", data, monkeypatch, **{zero: 0.0})
    lt, gt = _tape_step("fp32", "1", data, monkeypatch, **{zero: 0.0})
    key = {"ssim_weight": "coarse_ssim_loss", "vgg_weight": "coarse_vgg_loss"}[zero]
    assert la[key] == 0.0 and lt[key] == 0.0, (la[key], lt[key])
    assert abs(lt["loss_all"] - sum(v for k, v in lt.items() if k != "loss_all")) <= 1e-6 * abs(lt["loss_all"])
    for k in la:
        assert abs(la[k] - lt[k]) <= 1e-6 * max(1.0, abs(la[k])), (k, la[k], lt[k])
    errs = _rel(gt, ga)
    assert max(errs.values()) <= 1e-5, max(errs.values())


def test_adamax_matches_torch(dev):
    """Fused Adamax (flat-buffer and per-tensor paths) vs torch.optim.Adamax, 3 steps."""
    from deep_video_interpolation_extrapolation_amd.optim import Adamax
    g = torch.Generator().manual_seed(3)
    shapes = [(64, 3, 3, 3), (64,), (7, 5)]
    ref = [torch.randn(s, generator=g).requires_grad_(True) for s in shapes]
    mine = [r.detach().clone().to(dev).requires_grad_(True) for r in ref]
    o1 = torch.optim.Adamax(ref, lr=1e-3)
    o2 = Adamax(mine, lr=1e-3)
    for it in range(3):
        grads = [torch.randn(s, generator=g) * (10 ** -it) for s in shapes]
        for r, m, gg in zip(ref, mine, grads):
            r.grad = gg.clone()
            m.grad = gg.to(dev)
        o1.step()
        o2.step()
    for r, m in zip(ref, mine):
        assert float((m.detach().cpu() - r.detach()).abs().max()) < 1e-7
    sd = o2.state_dict()
    assert set(sd["state"][0].keys()) == {"step", "exp_avg", "exp_inf"}


def test_bf16_step_trains(dev):
    """bf16 mode: finite losses that decrease over a few steps on a fixed batch."""
    tr = trainer("bf16", 64, 128, 2)
    data = inputs.step_batch(2, 64, 128)
    losses = [float(tr.step(data)["loss_all"]) for _ in range(6)]
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses


def test_plan_reuse_and_busy_guard(dev):
    """A second forward while the first one's backward is pending gets its own plan."""
    tr = trainer("fp32", 32, 64, 2)
    m = tr.model.module
    x, seg = inputs.hrnet_input(2, 32, 64)
    r1, s1 = m(x.to(dev), seg.to(dev))
    r2, s2 = m(x.to(dev), seg.to(dev))
    assert torch.equal(r1, r2)
    (r1.sum() + r2.sum()).backward()
    n_plans = sum(len(v) for v in m.coarse_model._pool.plans.values())
    assert n_plans == 2


def test_main_launcher_one_epoch(dev, tmp_path):
    """The launcher (reference main.py flow): one training epoch on 2 synthetic clips, then
    the rank-0 checkpoint, then a validation pass reloading that checkpoint."""
    from deep_video_interpolation_extrapolation_amd import main as M
    common = ["--syn_type", "inter", "--bs", "2", "--input_h", "32", "--input_w", "64", "--epochs", "1",
              "--save_dir", str(tmp_path), "--synthetic", "2", "--nw", "0", "--precision", "fp32"]
    M.main(common + ["INTER", "--train_coarse"])
    runs = list(tmp_path.iterdir())
    assert len(runs) == 1
    ck = list((runs[0] / "checkpoint").iterdir())
    assert len(ck) == 1 and ck[0].name.startswith("InterNet_xs2xs_inter_0_1_")
    sd = torch.load(ck[0], map_location="cpu", weights_only=True)
    assert set(sd) == {"session", "epoch", "coarse_model", "coarse_opt"}
    M.main(common + ["--split", "val", "--load_dir", str(runs[0]), "--checkepoch", "1", "--checkpoint",
                          ck[0].name.split("_")[-1][:-4], "--checksession", "0", "INTER", "--load_coarse"])


def _head_grads(dev, im2col):
    os.environ["DVIE_IM2COL_DGRAD"] = "1" if im2col else "0"
    try:
        tr = trainer("bf16", 64, 128, 2)
        m = tr.model.module
        x, seg = inputs.hrnet_input(2, 64, 128)
        rgb, s = m(x.to(dev), seg.to(dev))
        g = torch.Generator().manual_seed(5)
        wr, ws = torch.randn(rgb.shape, generator=g).to(dev), torch.randn(s.shape, generator=g).to(dev)
        ((rgb * wr).sum() + (s * ws).sum()).backward()
        torch.cuda.synchronize()
        names = [getattr(o, "meta", {}).get("name", "") for pl in m.coarse_model._pool.plans.values()
                 for p in pl for o in getattr(p, "bwd", [])]
        return m.coarse_model._flat_grad.detach().float().clone(), names
    finally:
        os.environ.pop("DVIE_IM2COL_DGRAD", None)


def test_im2col_head_dgrad_matches_halo_path(dev):
    """bf16: the narrow-input head data gradients lowered to im2col + 1x1 GEMM give the same
    parameter gradients as the halo-kernel path (same products, different fp32 summation
    order: relative L2 within 1e-2 overall and per head-adjacent slice)."""
    g0, n0 = _head_grads(dev, False)
    g1, n1 = _head_grads(dev, True)
    assert not any(n.endswith(".im2col") for n in n0)
    assert sum(n.endswith(".im2col") for n in n1) == 2, [n for n in n1 if "im2col" in n]
    assert torch.isfinite(g1).all()
    rel = float((g1 - g0).norm() / g0.norm())
    assert rel < 1e-2, rel


def test_main_launcher_cycgen(dev, tmp_path):
    """--split cycgen (reference main.py:107-109, ExtraTrainer.py:586-679): one EXTRA
    training epoch on synthetic clips, then the rollout generation from a directory of
    rgb/seg PNG clips with the saved checkpoint: inputs + predictions written as rgb / seg /
    vis_seg PNGs at the input size."""
    from PIL import Image
    from deep_video_interpolation_extrapolation_amd import main as M
    common = ["--syn_type", "extra", "--bs", "2", "--input_h", "32", "--input_w", "64", "--epochs", "1",
              "--save_dir", str(tmp_path / "log"), "--synthetic", "2", "--nw", "0", "--precision", "fp32"]
    M.main(common + ["EXTRA", "--train_coarse"])
    run = next((tmp_path / "log").iterdir())
    ck = next((run / "checkpoint").iterdir())
    cyc = tmp_path / "cyc"
    rng = np.random.RandomState(0)
    for clip in ("aachen_000001", "bochum_000002"):
        for sub in ("rgb", "seg"):
            (cyc / sub / clip).mkdir(parents=True)
        for idx in ("00.0", "01.0"):
            Image.fromarray(rng.randint(0, 256, (32, 64, 3), dtype=np.uint8)).save(cyc / "rgb" / clip / f"{idx}.png")
            Image.fromarray(rng.randint(0, 20, (32, 64), dtype=np.uint8)).save(cyc / "seg" / clip / f"{idx}.png")
    M.main(common + ["--split", "cycgen", "--load_dir", str(run), "--checkepoch", "1", "--checkpoint",
                     ck.name.split("_")[-1][:-4], "--checksession", "0", "--cycgen_load_dir", str(cyc), "EXTRA",
                     "--load_coarse"])
    out = run / "cycgen" / "cityscape" / "32x64" / "extra_int_1_len_1_nearest"
    for sub in ("rgb", "seg", "vis_seg"):
        for clip in ("aachen_000001", "bochum_000002"):
            names = sorted(p.name for p in (out / sub / clip).iterdir())
            assert names == ["00.0.png", "01.0.png", "02.0.png"], (sub, clip, names)
            assert Image.open(out / sub / clip / "02.0.png").size == (64, 32)


def test_capturable_split_decided_when_a_param_has_no_grad(dev):
    """Capturable fused Adam (graph capture): a parameter without a gradient in the first
    eager step after set_capturable (SpectralNorm u / v before set_net_grad(True)) still fixes
    the group's 'step counts differ' decision on the host, so the captured step never reads
    device step counts; the replayed updates equal torch 1.0.1 Adam with per-parameter counts."""
    from deep_video_interpolation_extrapolation_amd.optim import Adam
    from oracle import disc as OD
    g = torch.Generator().manual_seed(5)
    p0 = [torch.randn(6, generator=g), torch.randn(3, generator=g)]
    ps = [t.clone().to(dev).requires_grad_(True) for t in p0]
    opt = Adam(ps, lr=1e-3)
    opt.set_capturable(True)
    g1 = [torch.randn(6, generator=g), torch.randn(3, generator=g)]
    ps[0].grad = g1[0].to(dev)  # ps[1] has no gradient: skipped, no state
    opt.step()
    assert opt._split == {0: True}
    ps[1].grad = g1[1].to(dev)
    opt.step()  # second eager step: ps[1] takes its first step here, outside the capture
    torch.cuda.synchronize()
    graph, side = torch.cuda.CUDAGraph(), torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph):
            opt.step()
    torch.cuda.current_stream(dev).wait_stream(side)
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    P = {0: p0[0].clone(), 1: p0[1].clone()}
    st = None
    for grads in ({0: g1[0]}, {0: g1[0], 1: g1[1]}, {0: g1[0], 1: g1[1]}, {0: g1[0], 1: g1[1]}):
        P, st = OD.adam_101(P, grads, 1e-3, st)
    for i in range(2):
        assert float((ps[i].detach().cpu() - P[i]).abs().max()) < 1e-6, i
