"""Generate the golden fixtures under tests/golden/ by running the REFERENCE code.

Run in the build container (it needs /root/reference; the GPU box does not have it):
    python tests/golden/make_golden.py
It imports the reference's own modules (nets, losses, utils.net_utils) read-only with the
offline stubs of ref_stubs.py and records their outputs on seeded inputs.  The fixtures are
data only (inputs are regenerated from seeds by tests/golden/inputs.py; outputs stored).

  hrnet_fwd.npz  G1: reference InterNet/HRNet forward, seed 1024, input (2,46,16,32)
                     + per-parameter checksums of the seeded initial weights
  rgbloss.npz    G2: reference RGBLoss components (+ d/dpred) on [-1,1] (normed=False,
                     as InterTrainer calls it) and [0,1] inputs; CE
  warp.npz       G3: reference FlowWrapper forward/backward (align_corners=True)
  metrics.npz    G5: reference PSNR / SSIM / IoU / VGGCosineLoss
  disc.npz       G6: reference FrameDiscriminator / VideoDiscriminator (seg_disc, BatchNorm
                     in train mode) at 128x128 and 128x256 (NCHW-flat head grouping): scores,
                     input gradients, parameter-gradient stats, running statistics, hinge
                     losses, eval-mode scores
  sepunet.npz    G7: reference SepUNet (train-mode BatchNorm, align_corners=True upsampling,
                     tanh head) at 32x64: outputs, input-gradient stats, parameter-gradient
                     stats, running statistics
  vaehrnet.npz   G9: reference VAEHRNet (train mode, 128x128): rgb / seg stats + samples, mu,
                     logvar, parameter-gradient stats, initial-weight checksums, running stats
  step.npz       G4: one training step of the reference modules (InterTrainer.py:380-441
                     body): loss dict, per-parameter gradient stats, post-Adamax checksums
  ckpt_manifest.json G10: the reference save_checkpoint dict (InterTrainer.py:867-885)
                     after the G4 step, written by torch.save and read back: its manifest
  refine.npz     G11/G12: reference InterRefineNet (SRNRefine) and InterStage3Net
                     (MSResAttnRefine, with / without stage3_prop), n_scales 2: outputs, flow
                     maps, parameter-gradient stats for seeded output gradients
  clip_crops.npz G13: reference get_seq_crop_params (folder.py:125-149) crops and the
                     flip draw (folder.py:211) for seeds 0..63
  gan_vae.npz    G14: two InterGANTrainer steps (runners/InterGANTrainer.py:376-456 body) of
                     the reference's own runnable InterGAN configuration: InterGANNet with a
                     VAEHRNet coarse model (KLD term) and FrameSN / VideoSN discriminators
                     (seg_disc), 128x128, batch 2; step 2 with SpectralNorm u / v trainable
                     (set_net_grad(True)): loss dicts, gradient stats, post-step checksums, u / v,
                     BatchNorm running statistics, 64 seeded elements of every gradient and every
                     post-step tensor, the post-step values of the BatchNorm-preceding biases
  gan_vae64.npz  G14d: the same two steps with the reference modules widened to float64 after
                     their seeded fp32 initialisation (float64 draws after that), the same
                     records plus step 1's near-zero gradient elements (index, value)
"""
import os
import sys
import types
import warnings

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
warnings.filterwarnings("ignore")

import inputs  # noqa: E402
import ref_stubs  # noqa: E402
from oracle.losses import synthetic_vgg19_state  # noqa: E402

ref_stubs.install(synthetic_vgg19_state)
import losses as ref_losses  # noqa: E402  (reference losses.py)
import nets as ref_nets  # noqa: E402      (reference nets/)
from utils import net_utils as ref_nu  # noqa: E402

torch.set_num_threads(8)


def args_ns(**kw):
    a = types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet", num_pred_once=1,
                              inpaint=False, inpaint_mask=False, fix_init_frames=False, l1_weight=80.0,
                              gdl_weight=80.0, vgg_weight=20.0, ssim_weight=20.0, ce_weight=30.0, vid_length=1)
    a.__dict__.update(kw)
    return a


def checksums(sd):
    names = sorted(sd)
    return names, np.array([[float(sd[n].double().sum()), float((sd[n].double() ** 2).sum())] for n in names])


def g1():
    torch.manual_seed(1024)
    model = ref_nets.InterNet(args_ns())
    x, seg = inputs.hrnet_input(2, 16, 32)
    with torch.no_grad():
        rgb, segout = model(x, seg=seg)
    names, cs = checksums(model.coarse_model.state_dict())
    np.savez_compressed(os.path.join(HERE, "hrnet_fwd.npz"), rgb=rgb.numpy(), seg=segout.numpy(),
                        param_names=np.array(names), param_checksums=cs,
                        n_params=sum(p.numel() for p in model.parameters()))


def g2():
    out = {}
    for tag, (pred, gt, normed) in inputs.rgbloss_inputs().items():
        loss = ref_losses.RGBLoss(args_ns())
        pred = pred.clone().requires_grad_(True)
        d = loss(pred, gt, normed, prefix="coarse")
        for k, v in d.items():
            (g,) = torch.autograd.grad(v, pred, retain_graph=True)
            key = k.replace("coarse_", "")
            out[f"{tag}_{key}"] = np.float64(v.item())
            out[f"{tag}_{key}_grad"] = g.numpy()
    logits, onehot = inputs.ce_inputs()
    logits = logits.clone().requires_grad_(True)
    ce = torch.nn.CrossEntropyLoss()(logits, torch.argmax(onehot, dim=1))
    (g,) = torch.autograd.grad(ce, logits)
    out["ce"] = np.float64(ce.item())
    out["ce_grad"] = g.numpy()
    np.savez_compressed(os.path.join(HERE, "rgbloss.npz"), **out)


def g3():
    x, flow, dout = inputs.warp_inputs()
    x = x.clone().requires_grad_(True)
    flow = flow.clone().requires_grad_(True)
    y = ref_nu.FlowWrapper()(x, flow)
    gx, gf = torch.autograd.grad(y, (x, flow), dout)
    np.savez_compressed(os.path.join(HERE, "warp.npz"), out=y.detach().numpy(), dx=gx.numpy(), dflow=gf.numpy())


def g5():
    pred, gt = inputs.metric_inputs()
    psnr = ref_losses.PSNR()(pred, gt)
    ssim = ref_losses.SSIM()(pred, gt)
    a, b = inputs.iou_inputs()
    iou = ref_losses.IoU()(a, b)
    vcos = ref_losses.VGGCosineLoss()(pred * 2 - 1, gt * 2 - 1, normed=False)
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), psnr=psnr.item(), ssim=ssim.item(), iou=iou.item(),
                        vgg_cos=vcos.item())


def g4():
    args = args_ns()
    torch.manual_seed(1024)
    model = ref_nets.InterNet(args)
    rgb_loss = ref_losses.RGBLoss(args)
    ce = torch.nn.CrossEntropyLoss()
    opt = torch.optim.Adamax(list(model.coarse_model.parameters()), lr=1e-3)
    data = inputs.step_batch(2, 32, 64)
    # runners/InterTrainer.py:389-437 (W = 1: sync is the identity)
    gt_x = data["frame2"]
    gt_seg = data["seg2"]
    x = torch.cat([data["frame1"], data["frame3"]], dim=1)
    seg = torch.cat([data["seg1"], data["seg3"]], dim=1)
    coarse_img, coarse_seg = model(x, seg=seg)
    loss_dict = rgb_loss(coarse_img, gt_x, False, prefix="coarse")
    loss_dict["coarse_ce_loss"] = args.ce_weight * ce(coarse_seg, torch.argmax(gt_seg, dim=1))
    loss = 0
    for v in loss_dict.values():
        loss += torch.mean(v)
    loss_dict["loss_all"] = loss
    opt.zero_grad()
    loss_dict["loss_all"].backward()
    named = dict(model.coarse_model.named_parameters())
    names = sorted(named)
    gstats = np.array([[float(named[n].grad.double().sum()), float((named[n].grad.double() ** 2).sum()),
                        float(named[n].grad.abs().max())] for n in names])
    opt.step()
    _, post = checksums({n: p.detach() for n, p in named.items()})
    np.savez_compressed(os.path.join(HERE, "step.npz"), loss_names=np.array(list(loss_dict.keys())),
                        loss_values=np.array([float(v) for v in loss_dict.values()]), param_names=np.array(names),
                        grad_stats=gstats, post_checksums=post, rgb=coarse_img.detach().numpy()[:, :, ::4, ::4],
                        seg=coarse_seg.detach().numpy()[:, :, ::4, ::4])


def g6():
    out = {}
    for tag, cls, seed in (("frame", "FrameDiscriminator", 31), ("video", "VideoDiscriminator", 32)):
        for H, W in ((128, 128), (128, 256)):
            t = f"{tag}_{H}x{W}"
            torch.manual_seed(seed)
            d = ref_nets.__dict__[cls](args_ns(seg_disc=True))
            d.train()
            x, seg, ix, iseg, gout = inputs.disc_inputs(2, H, W)
            ins = [x, seg] + ([ix, iseg] if tag == "video" else [])
            ins = [v.clone().requires_grad_(True) for v in ins]
            score = d(*ins)
            score.backward(gout)
            out[t + "_score"] = score.detach().numpy()
            for k, v in enumerate(ins):  # large: stats + seeded sample points (inputs.sample_idx)
                gv = v.grad.double().reshape(-1)
                out[t + f"_gin{k}"] = np.concatenate([[float(gv.sum()), float(gv.abs().sum()), float(gv.norm())],
                                                      gv[inputs.sample_idx(gv.numel())].numpy()])
            named = dict(d.named_parameters())
            names = sorted(named)
            out[t + "_param_names"] = np.array(names)
            out[t + "_grad_stats"] = np.array([[float(named[n].grad.double().sum()),
                                                float((named[n].grad.double() ** 2).sum())] for n in names])
            bufs = {k: v for k, v in d.state_dict().items() if "running" in k}
            out[t + "_buf_names"] = np.array(sorted(bufs))
            out[t + "_bufs"] = np.concatenate([bufs[k].numpy() for k in sorted(bufs)])
            gl = ref_losses.GANScalarLoss(weight=1.5)
            out[t + "_hinge"] = np.array([gl(score, True).item(), gl(score, False).item()])
            d.eval()
            with torch.no_grad():
                out[t + "_score_eval"] = d(*[v.detach() for v in ins]).numpy()
    np.savez_compressed(os.path.join(HERE, "disc.npz"), **out)


def g7():
    torch.manual_seed(5)
    m = ref_nets.SepUNet(args_ns())
    m.train()
    inp, mask, g_rgb, g_seg = inputs.sepunet_inputs()
    inp = inp.clone().requires_grad_(True)
    rgb, seg = m(inp, fg_mask=mask)
    (rgb * g_rgb).sum().add((seg * g_seg).sum()).backward()
    named = dict(m.named_parameters())
    names = sorted(named)
    gi = inp.grad.double().reshape(-1)
    bufs = {k: v for k, v in m.state_dict().items() if "running" in k}
    np.savez_compressed(os.path.join(HERE, "sepunet.npz"), rgb=rgb.detach().numpy(), seg=seg.detach().numpy(),
                        gin=np.concatenate([[float(gi.sum()), float(gi.abs().sum()), float(gi.norm())],
                                            gi[inputs.sample_idx(gi.numel())].numpy()]),
                        param_names=np.array(names),
                        grad_stats=np.array([[float(named[n].grad.double().sum()),
                                              float((named[n].grad.double() ** 2).sum())] for n in names]),
                        buf_names=np.array(sorted(bufs)),
                        bufs=np.concatenate([bufs[k].numpy().reshape(-1) for k in sorted(bufs)]))


G8_CASES = (("FrameLocalDiscriminator", 51), ("FrameSNDiscriminator", 52), ("FrameSNLocalDiscriminator", 53),
            ("VideoLocalDiscriminator", 54), ("VideoSNDiscriminator", 55), ("VideoSNLocalDiscriminator", 56))


def g8():
    """the remaining discriminator variants (local map outputs, SpectralNorm) at 128x128,
    seg_disc, train mode: one forward + backward each; `uvgrad` repeats the SN ones with every
    parameter requiring grad (the state after InterGANNet's set_net_grad(True))."""
    out = {}
    for cls, seed in G8_CASES:
        for uvgrad in ((False, True) if "SN" in cls else (False,)):
            t = cls + ("_uvgrad" if uvgrad else "")
            torch.manual_seed(seed)
            d = ref_nets.__dict__[cls](args_ns(seg_disc=True))
            d.train()
            if uvgrad:
                for p in d.parameters():
                    p.requires_grad = True
            x, seg, ix, iseg, gout = inputs.disc_inputs(2, 128, 128)
            ins = [x, seg] + ([ix, iseg] if cls.startswith("Video") else [])
            ins = [v.clone().requires_grad_(True) for v in ins]
            score = d(*ins)
            if score.dim() > 1:
                gout = inputs.disc_map_grad(tuple(score.shape))
            score.backward(gout)
            out[t + "_score"] = score.detach().numpy()
            for k, v in enumerate(ins):
                gv = v.grad.double().reshape(-1)
                out[t + f"_gin{k}"] = np.concatenate([[float(gv.sum()), float(gv.abs().sum()), float(gv.norm())],
                                                      gv[inputs.sample_idx(gv.numel())].numpy()])
            named = dict(d.named_parameters())
            names = sorted(n for n in named if named[n].grad is not None)
            out[t + "_param_names"] = np.array(names)
            out[t + "_grad_stats"] = np.array([[float(named[n].grad.double().sum()),
                                                float((named[n].grad.double() ** 2).sum())] for n in names])
            sd = d.state_dict()
            uv = sorted(k for k in sd if k.endswith("weight_u") or k.endswith("weight_v"))
            if uv:  # u, v after the forward's power iteration
                out[t + "_uv_names"] = np.array(uv)
                out[t + "_uv"] = np.concatenate([sd[k].numpy().reshape(-1) for k in uv])
            bufs = {k: v for k, v in sd.items() if "running" in k}
            if bufs:
                out[t + "_buf_names"] = np.array(sorted(bufs))
                out[t + "_bufs"] = np.concatenate([bufs[k].numpy() for k in sorted(bufs)])
    np.savez_compressed(os.path.join(HERE, "disc_sn.npz"), **out)


def g9():
    """reference VAEHRNet (train mode, 128x128 - its only working size) forward + backward:
    the reparameterisation noise is the CPU draw right after torch.manual_seed(77)"""
    torch.manual_seed(1024)
    m = ref_nets.VAEHRNet(args_ns())
    m.train()
    x, seg, gt_x, gt_seg, (g_rgb, g_seg, g_mu, g_lv) = inputs.vae_inputs()
    torch.manual_seed(77)
    rgb, segout, mu, logvar = m(torch.cat([x, seg], 1), gt_x, gt_seg)
    ((rgb * g_rgb).sum() + (segout * g_seg).sum() + (mu * g_mu).sum() + (logvar * g_lv).sum()).backward()
    out = {"mu": mu.detach().numpy(), "logvar": logvar.detach().numpy()}
    for k, t in (("rgb", rgb), ("seg", segout)):
        v = t.detach().double().reshape(-1)
        out[k] = np.concatenate([[float(v.sum()), float(v.abs().sum()), float(v.norm())],
                                 v[inputs.sample_idx(v.numel())].numpy()])
    named = dict(m.named_parameters())
    names = sorted(named)
    out["param_names"] = np.array(names)
    out["grad_stats"] = np.array([[float(named[n].grad.double().sum()), float((named[n].grad.double() ** 2).sum())]
                                  for n in names])
    _, cs = checksums({n: p.detach() for n, p in named.items()})
    out["param_checksums"] = cs
    bufs = {k: v for k, v in m.state_dict().items() if "running" in k}
    out["buf_names"] = np.array(sorted(bufs))
    out["bufs"] = np.concatenate([bufs[k].numpy().reshape(-1) for k in sorted(bufs)])
    np.savez_compressed(os.path.join(HERE, "vaehrnet.npz"), **out)


def _tstat(t):
    t = t.detach()
    return {"dtype": str(t.dtype).replace("torch.", ""), "shape": list(t.shape),
            "sum": float(t.double().sum()), "sumsq": float((t.double() ** 2).sum())}


def g10():
    """Checkpoint format (reference runners/InterTrainer.py:867-885 save_checkpoint): the
    reference modules take the G4 training step, then the reference's save_dict is written
    with torch.save and read back.  The file itself is ~120 MB (9.9 M fp32 weights + two
    Adamax state tensors each), so the fixture is its manifest: top-level keys and values,
    every state_dict entry in order with dtype / shape / sum / sum of squares, and the
    optimizer state_dict's param_groups and per-index state the same way.  Tests rebuild
    the file from the oracle step (pinned by G4) and check it against this manifest before
    loading it."""
    import json
    import tempfile
    args = args_ns()
    torch.manual_seed(1024)
    model = ref_nets.InterNet(args)
    rgb_loss = ref_losses.RGBLoss(args)
    ce = torch.nn.CrossEntropyLoss()
    coarse_opt = torch.optim.Adamax(list(model.coarse_model.parameters()), lr=1e-3)
    data = inputs.step_batch(2, 32, 64)
    x = torch.cat([data["frame1"], data["frame3"]], dim=1)
    seg = torch.cat([data["seg1"], data["seg3"]], dim=1)
    coarse_img, coarse_seg = model(x, seg=seg)
    ld = rgb_loss(coarse_img, data["frame2"], False, prefix="coarse")
    ld["coarse_ce_loss"] = args.ce_weight * ce(coarse_seg, torch.argmax(data["seg2"], dim=1))
    loss = 0
    for v in ld.values():
        loss += torch.mean(v)
    coarse_opt.zero_grad()
    loss.backward()
    coarse_opt.step()
    # save_checkpoint (session 1, epoch 1 -> 'epoch': 2, step 0)
    save_dict = {"session": 1, "epoch": 1 + 1, "coarse_model": model.coarse_model.state_dict(),
                 "coarse_opt": coarse_opt.state_dict()}
    name = "{}_{}_{}_{}".format("InterNet", "xs2xs", "inter", 1) + "_{}_{}.pth".format(1, 0)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, name)
        torch.save(save_dict, path)
        ck = torch.load(path, map_location="cpu", weights_only=True)
    man = {"file": name, "top_keys": list(ck.keys()), "session": ck["session"], "epoch": ck["epoch"],
           "coarse_model": [[k, _tstat(v)] for k, v in ck["coarse_model"].items()],
           "coarse_opt": {"param_groups": [{k: v for k, v in g.items()} for g in ck["coarse_opt"]["param_groups"]],
                          "state": {str(i): {k: (_tstat(v) if torch.is_tensor(v) else v) for k, v in st.items()}
                                    for i, st in ck["coarse_opt"]["state"].items()}}}
    with open(os.path.join(HERE, "ckpt_manifest.json"), "w") as f:
        json.dump(man, f, indent=0, sort_keys=False)


def _gstats(module):
    named = dict(module.named_parameters())
    names = sorted(n for n in named if named[n].grad is not None)
    return np.array(names), np.array([[float(named[n].grad.double().sum()), float((named[n].grad.double() ** 2).sum())]
                                      for n in names])


def _samples(module_or_sd, names, grad):
    """64 seeded elements of each named gradient (grad=True) or state tensor, in names order
    (inputs.sample_idx(numel, 64): fixed positions per tensor size)"""
    src = dict(module_or_sd.named_parameters()) if grad else module_or_sd
    rows = []
    for n in names:
        t = src[str(n)].grad if grad else src[str(n)]
        v = t.detach().double().reshape(-1)
        rows.append(v[inputs.sample_idx(v.numel(), 64)].numpy())
    return np.array(rows)


def _small_grads(module, names, rel=1e-5):
    """(tensor index, flat index, value) of every gradient element with 0 < |g| <= rel * max|g| of
    its tensor: the elements whose sign rounding can decide (Adamax / Adam take a first step of
    +-lr whatever |g| is), so a check can start its next step from the reference's own signs"""
    named = dict(module.named_parameters())
    rows = []
    for i, n in enumerate(names):
        g = named[str(n)].grad.detach().double().reshape(-1)
        m = (g != 0) & (g.abs() <= rel * float(g.abs().max()))
        idx = torch.nonzero(m).reshape(-1)
        rows += [[i, int(j), float(g[j])] for j in idx]
    return np.array(rows, dtype=np.float64).reshape(-1, 3)


def _flat_sample(t):
    v = t.detach().double().reshape(-1)
    return np.concatenate([[float(v.sum()), float(v.abs().sum()), float(v.norm())],
                           v[inputs.sample_idx(v.numel())].numpy()])


def g11():
    """reference InterRefineNet (HRNet coarse + SRNRefine, n_scales 2; nets/InterRefineNet.py:8-28,
    nets/refine_nets.py:27-135), train split, 32x64: forward outputs, and the refine net's
    parameter gradients for seeded upstream gradients of every refine output; and G12:
    InterStage3Net (+ MSResAttnRefine, refine_nets.py:138-399) at 64x128 with and without
    stage3_prop: outputs, flow maps, stage-3 parameter gradients."""
    out = {}
    for tag, cls, H, W, prop in (("refine", "InterRefineNet", 32, 64, False), ("stage3", "InterStage3Net", 64, 128, False),
                                 ("stage3prop", "InterStage3Net", 64, 128, True)):
        args = args_ns(refine_model="SRNRefine", stage3_model="MSResAttnRefine", n_scales=2, split="train",
                       with_gt_seg=False, stage3_prop=prop)
        torch.manual_seed(1024)
        m = ref_nets.__dict__[cls](args)
        x, seg = inputs.hrnet_input(2, H, W)
        res = m(x, seg=seg)
        g = torch.Generator().manual_seed(91)
        outs = list(res[2]) + (list(res[3]) if cls == "InterStage3Net" else [])
        loss = sum((o * torch.randn(o.shape, generator=g)).sum() for o in outs)
        loss.backward()
        small = cls == "InterRefineNet"  # the 64x128 outputs are stored as stats + seeded samples
        for i, o in enumerate(res[2]):
            out[f"{tag}_refine{i}"] = o.detach().numpy() if small else _flat_sample(o)
        if cls == "InterStage3Net":
            for i, o in enumerate(res[3]):
                out[f"{tag}_stage3_{i}"] = _flat_sample(o)
            for i, f in enumerate(res[4]):
                out[f"{tag}_flow{i}"] = f.numpy()
            out[f"{tag}_names"], out[f"{tag}_grad_stats"] = _gstats(m.stage3_model)
        out[f"{tag}_refine_names"], out[f"{tag}_refine_grad_stats"] = _gstats(m.refine_model)
        _, out[f"{tag}_refine_init"] = checksums({k: v for k, v in m.refine_model.state_dict().items()})
    np.savez_compressed(os.path.join(HERE, "refine.npz"), **out)


def g12():
    """reference folder.py:125-149 get_seq_crop_params (the pseudo-motion crops of the
    Cityscapes clip loader; it reads no instance state) for np.random seeds 0..63, and the
    horizontal-flip draw of folder.py:211 (random.randint(0, 2)) for random seeds 0..63."""
    import random
    import folder as ref_folder  # reference folder.py
    cls = next(v for v in vars(ref_folder).values() if isinstance(v, type) and hasattr(v, "get_seq_crop_params"))
    crops, flips = [], []
    for seed in range(64):
        np.random.seed(seed)
        crops.append([list(c) for c in cls.get_seq_crop_params(None)])
        random.seed(seed)
        flips.append(ref_folder.randint(0, 2))
    np.savez_compressed(os.path.join(HERE, "clip_crops.npz"), crops=np.array(crops), flips=np.array(flips))


def g14(dtype=torch.float32, fname="gan_vae.npz"):
    """The reference's InterGAN step body composed from its own modules (InterGANNet forward,
    RGBLoss on (x + 1) / 2, 30 * CrossEntropy, KLDLoss, GANScalarLoss, Adamax / Adam), W = 1.
    The reparameterisation noise of step k is the CPU draw right after torch.manual_seed(78 + k)
    (inputs.vae_eps(2, 78 + k)): the coarse model's reparameterize is the forward's first RNG use.
    `Tensor.cuda` is the identity here (InterGANNet.py:35 moves a zero tensor to the GPU)."""
    args = args_ns(coarse_model="VAEHRNet", frame_disc=True, video_disc=True, frame_det_disc=False,
                   video_det_disc=False, track_gen=False, frame_disc_model="FrameSNDiscriminator",
                   video_disc_model="VideoSNDiscriminator", seg_disc=True, rank=0, kld_weight=20.0, vae=True)
    cuda0 = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    dt0 = torch.get_default_dtype()
    try:
        torch.manual_seed(1024)
        model = ref_nets.InterGANNet(args)
        if dtype != torch.float32:  # float64 run (G14d): the same seeded fp32 init, then widened
            torch.set_default_dtype(dtype)
            model = model.to(dtype)
        model.train()
        rgb_loss = ref_losses.RGBLoss(args)
        kld = ref_losses.KLDLoss(args)
        ce = torch.nn.CrossEntropyLoss()
        d_loss, g_loss = ref_losses.GANScalarLoss(weight=1.0), ref_losses.GANScalarLoss(weight=1.0)
        coarse_opt = torch.optim.Adamax(list(model.coarse_model.parameters()), lr=1e-3)
        frame_opt = torch.optim.Adam(list(model.frame_disc_model.parameters()), lr=1e-3)
        video_opt = torch.optim.Adam(list(model.video_disc_model.parameters()), lr=1e-3)
        out = {}
        for mod, tag in ((model.coarse_model, "g"), (model.frame_disc_model, "f"), (model.video_disc_model, "v")):
            out[tag + "_init_names"], out[tag + "_init"] = checksums(dict(mod.state_dict()))
        data = inputs.step_batch(2, 128, 128)
        data = {k: (v.to(dtype) if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in data.items()}
        for k in range(2):
            gt_x, gt_seg = data["frame2"], data["seg2"]
            x = torch.cat([data["frame1"], data["frame3"]], dim=1)
            seg = torch.cat([data["seg1"], data["seg3"]], dim=1)
            torch.manual_seed(78 + k)
            res = model(x, seg, gt_x, gt_seg, bboxes=data.get("bboxes"))
            coarse_img, coarse_seg, mu, logvar = res[:4]
            dff, drf, dfv, drv, gff, gfv = res[4:10]
            norm = lambda t: (t + 1) / 2  # noqa: E731  InterGANTrainer.normalize
            ld = rgb_loss(norm(coarse_img), norm(gt_x), False, prefix="coarse")
            ld["coarse_ce_loss"] = args.ce_weight * ce(coarse_seg, torch.argmax(gt_seg, dim=1))
            ld["coarse_kld_loss"] = kld(mu, logvar)
            ld["coarse_frame_loss"] = g_loss(gff, True)
            ld["disc_frame_real_loss"] = d_loss(drf, True)
            ld["disc_frame_fake_loss"] = d_loss(dff, False)
            ld["coarse_video_loss"] = g_loss(gfv, True)
            ld["disc_video_real_loss"] = d_loss(drv, True)
            ld["disc_video_fake_loss"] = d_loss(dfv, False)
            loss = 0
            for v in ld.values():
                loss += torch.mean(v)
            ld["loss_all"] = loss
            for o in (coarse_opt, frame_opt, video_opt):
                o.zero_grad()
            loss.backward()
            t = f"step{k + 1}_"
            out[t + "loss_names"] = np.array(list(ld.keys()))
            out[t + "loss_values"] = np.array([float(v) for v in ld.values()])
            for mod, tag in ((model.coarse_model, "g"), (model.frame_disc_model, "f"), (model.video_disc_model, "v")):
                out[t + tag + "_grad_names"], out[t + tag + "_grad_stats"] = _gstats(mod)
                out[t + tag + "_grad_samples"] = _samples(mod, out[t + tag + "_grad_names"], True)
                if dtype != torch.float32 and k == 0:
                    out[t + tag + "_grad_small"] = _small_grads(mod, out[t + tag + "_grad_names"])
            for o in (coarse_opt, frame_opt, video_opt):
                o.step()
            for mod, tag in ((model.coarse_model, "g"), (model.frame_disc_model, "f"), (model.video_disc_model, "v")):
                out[t + tag + "_post_names"], out[t + tag + "_post"] = checksums(dict(mod.state_dict()))
                sd = dict(mod.state_dict())
                out[t + tag + "_post_samples"] = _samples(sd, out[t + tag + "_post_names"], False)
            # the conv biases right before a train-mode BatchNorm get a rounding-noise gradient (true
            # value 0) that Adamax turns into +-lr steps: their whole post-step values, so a check of
            # the next step can start from the reference's own
            sd = dict(model.coarse_model.state_dict())
            bn_b = sorted(n for n in sd if n.endswith(".bias") and "." in n[:-5] and n[:-5].rsplit(".", 1)[1].isdigit()
                          and f"{n[:-5].rsplit('.', 1)[0]}.{int(n[:-5].rsplit('.', 1)[1]) + 1}.running_mean" in sd)
            out[t + "g_bnbias_names"] = np.array(bn_b)
            out[t + "g_bnbias_post"] = np.concatenate([sd[n].detach().double().reshape(-1).numpy() for n in bn_b])
        np.savez_compressed(os.path.join(HERE, fname), **out)
    finally:
        torch.Tensor.cuda = cuda0
        torch.set_default_dtype(dt0)


def g14d():
    """G14 in float64 (gan_vae64.npz): the same two steps with the reference modules widened to
    float64 after their seeded fp32 initialisation, so a per-tensor comparison with the float64
    oracle sees the algorithm, not fp32 rounding (which the VAE decoder's gradients amplify about
    100x by the second step: the oracle's own fp32 and fp64 runs differ by 2.4e-4 there)."""
    g14(torch.float64, "gan_vae64.npz")


if __name__ == "__main__":
    import sys as _sys
    todo = {f.__name__: f for f in (g1, g2, g3, g5, g4, g6, g7, g8, g9, g10, g11, g12, g14, g14d)}
    for name in (_sys.argv[1:] or list(todo)):
        f = todo[name]
        f()
        print("wrote", f.__name__)
