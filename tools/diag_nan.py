"""Run bench-shaped InterTrainer steps and report the first non-finite loss / gradient
(which parameters), to localise a kernel producing NaN/Inf at full size.
    python tools/diag_nan.py [steps] [H] [W] [batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    os.environ["DVIE_PRECISION"] = "bf16"
    dev = torch.device("cuda", 0)
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer
    args = default_args("INTER", syn_type="inter", mode="xs2xs", interval=5, vid_length=1, train_coarse=True,
                        batch_size=B, input_h=H, input_w=W, precision="bf16", synthetic=B, num_workers=0,
                        split="train", rank=0, gpus=1)
    torch.manual_seed(args.seed)
    tr = InterTrainer(args)
    data = bench.make_batch(B, H, W, dev, 0)
    named = list(tr.model.module.coarse_model.named_parameters())
    from deep_video_interpolation_extrapolation_amd import engine
    trace_from = int(os.environ.get("TRACE_FROM", "-1"))
    for s in range(steps):
        engine.DEBUG_NAN = s >= trace_from >= 0
        if os.environ.get("TERMS_AT") == str(s):
            loss_terms(tr, data)
        ld = tr.step(data)
        torch.cuda.synchronize()
        print(f"step {s}: " + " ".join(f"{k}={float(v):.4g}" for k, v in ld.items()), flush=True)
        bad = [(n, p.grad) for n, p in named if p.grad is not None and not torch.isfinite(p.grad).all()]
        badp = [n for n, p in named if not torch.isfinite(p.data).all()]
        if bad or badp:
            print(f"  non-finite grads in {len(bad)} params, non-finite values in {len(badp)} params")
            for n, g in bad[:40]:
                print(f"   grad {n} {tuple(g.shape)} nan={int(torch.isnan(g).sum())} inf={int(torch.isinf(g).sum())}")
            for n in badp[:10]:
                print(f"   value {n}")
            break


def loss_terms(tr, data):
    """Per-loss-term finiteness of d(term)/d(prediction) at the trainer's current weights."""
    from deep_video_interpolation_extrapolation_amd.data import batch_to
    data = batch_to(data, tr.device)
    x, seg, gt_x, gt_seg = tr.get_input(data)
    img, segout = tr.model(x, seg=seg)
    img_d = img.detach().requires_grad_(True)
    seg_d = segout.detach().requires_grad_(True)
    rl = tr.RGBLoss
    terms = {"l1": lambda: rl.l1_loss(img_d, gt_x), "gdl": lambda: rl.gdl_loss(img_d, gt_x),
             "ssim": lambda: rl.ssim_loss(img_d, gt_x), "vgg": lambda: rl.vgg_loss(img_d, gt_x, False)}
    print(f"  pred finite {bool(torch.isfinite(img).all())} seg finite {bool(torch.isfinite(segout).all())} "
          f"pred range [{float(img.min()):.3g}, {float(img.max()):.3g}]")
    for k, f in terms.items():
        v = f()
        (g,) = torch.autograd.grad(v.mean(), img_d)
        print(f"  {k}: value {float(v.mean()):.4g} grad finite {bool(torch.isfinite(g).all())} "
              f"nan {int(torch.isnan(g).sum())}")
    ce = tr.SegLoss(seg_d, gt_seg)
    (g,) = torch.autograd.grad(ce.mean(), seg_d)
    print(f"  ce: value {float(ce.mean()):.4g} grad finite {bool(torch.isfinite(g).all())}")


if __name__ == "__main__":
    main()
