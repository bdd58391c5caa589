"""Seeded inputs of the golden fixtures (shared by make_golden.py and the tests)."""
import torch


def _gen(seed):
    return torch.Generator().manual_seed(seed)


def onehot(lab, n=20):
    return torch.nn.functional.one_hot(lab, n).permute(0, 3, 1, 2).float()


def hrnet_input(n, H, W, seed=7):
    g = _gen(seed)
    x = torch.rand((n, 6, H, W), generator=g) * 2 - 1
    seg = torch.cat([onehot(torch.randint(0, 20, (n, H, W), generator=g)) for _ in range(2)], 1)
    return x, seg


def rgbloss_inputs():
    g = _gen(11)
    pred = torch.rand((2, 3, 16, 32), generator=g) * 2 - 1
    gt = (torch.rand((2, 3, 16, 32), generator=g) * 2 - 1) * 0.7 + 0.2 * pred
    g01 = _gen(12)
    p01 = torch.rand((2, 3, 16, 32), generator=g01)
    t01 = torch.rand((2, 3, 16, 32), generator=g01) * 0.6 + 0.3 * p01
    return {"pm1": (pred, gt, False), "z1": (p01, t01, False), "normed": (pred, gt, True)}


def ce_inputs():
    g = _gen(13)
    logits = torch.randn((2, 20, 16, 32), generator=g) * 3
    lab = torch.randint(0, 20, (2, 16, 32), generator=g)
    return logits, onehot(lab)


def warp_inputs():
    g = _gen(17)
    x = torch.rand((2, 3, 16, 20), generator=g)
    flow = (torch.rand((2, 2, 16, 20), generator=g) * 2 - 1) * 0.6  # reaches outside the image
    dout = torch.randn((2, 3, 16, 20), generator=g)
    return x, flow, dout


def metric_inputs():
    g = _gen(19)
    pred = torch.rand((2, 3, 32, 64), generator=g)
    gt = (pred + 0.1 * torch.randn((2, 3, 32, 64), generator=g)).clamp(0, 1)
    return pred, gt


def iou_inputs():
    g = _gen(23)
    a = torch.randint(0, 20, (2, 32, 64), generator=g)
    b = torch.where(torch.rand((2, 32, 64), generator=g) < 0.7, a, torch.randint(0, 20, (2, 32, 64), generator=g))
    return a, b


def step_batch(n, H, W):
    out = {f"frame{k}": [] for k in (1, 2, 3)}
    out.update({f"seg{k}": [] for k in (1, 2, 3)})
    for i in range(n):
        g = _gen(1000 + i)
        for k in (1, 2, 3):
            out[f"frame{k}"].append(torch.rand((3, H, W), generator=g) * 2 - 1)
        for k in (1, 2, 3):
            lab = torch.randint(0, 20, (H, W), generator=g)
            out[f"seg{k}"].append(torch.nn.functional.one_hot(lab, 20).permute(2, 0, 1).float())
    return {k: torch.stack(v) for k, v in out.items()}


def disc_inputs(n=2, H=128, W=256, seed=21):
    """frame disc (x, seg) and video disc extra (input_x, input_seg); upstream score grads."""
    g = _gen(seed)
    x = torch.rand((n, 3, H, W), generator=g) * 2 - 1
    seg = torch.softmax(torch.randn((n, 20, H, W), generator=g) * 2, dim=1)
    ix = torch.rand((n, 6, H, W), generator=g) * 2 - 1
    iseg = torch.cat([onehot(torch.randint(0, 20, (n, H, W), generator=g)) for _ in range(2)], 1)
    k = (H // 128) * (W // 128)
    gout = torch.randn((n * k,), generator=g)
    return x, seg, ix, iseg, gout


def disc_map_grad(shape, seed=27):
    """upstream gradient of a local (map-output) discriminator"""
    return torch.randn(shape, generator=_gen(seed))


def sample_idx(numel, k=256, seed=99):
    """fixed sample positions for large-tensor fixtures"""
    return torch.randint(0, numel, (k,), generator=_gen(seed))


def sepunet_inputs(n=2, H=32, W=64, seed=41):
    """SepUNet input [frames 6 | segs 40], fg_mask (n, 2, H, W) in [0, 1], output grads."""
    g = _gen(seed)
    x = torch.rand((n, 6, H, W), generator=g) * 2 - 1
    seg = torch.cat([onehot(torch.randint(0, 20, (n, H, W), generator=g)) for _ in range(2)], 1)
    mask = (torch.rand((n, 2, H, W), generator=g) > 0.5).float() * 0.8 + 0.1
    g_rgb = torch.randn((n, 3, H, W), generator=g)
    g_seg = torch.randn((n, 20, H, W), generator=g)
    return torch.cat([x, seg], 1), mask, g_rgb, g_seg


def vae_inputs(n=2, H=128, W=128, seed=61):
    """VAEHRNet: frames / segs (hrnet_input), gt frame + one-hot seg, and upstream gradients of
    (rgb, seg, mu, logvar)."""
    x, seg = hrnet_input(n, H, W)
    g = _gen(seed)
    gt_x = torch.rand((n, 3, H, W), generator=g) * 2 - 1
    gt_seg = onehot(torch.randint(0, 20, (n, H, W), generator=g))
    grads = (torch.randn((n, 3, H, W), generator=g), torch.randn((n, 20, H, W), generator=g),
             torch.randn((n, 1024), generator=g), torch.randn((n, 1024), generator=g))
    return x, seg, gt_x, gt_seg, grads


def vae_eps(n=2, seed=77):
    """the reparameterisation noise the reference draws right after torch.manual_seed(seed)
    (std.new(std.size()).normal_(), nets/HRNet.py:963)"""
    torch.manual_seed(seed)
    return torch.empty(n, 1024).normal_()
