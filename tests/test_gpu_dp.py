"""GPU: data-parallel equivalence of the trainer step at world size 2 (two processes on
the one GPU, gloo over device tensors) against one process on the concatenated batch.

Reference semantics (runners/InterTrainer.py:431-436, 859-864; DDP): each rank back-props
loss_all / W and DDP averages, so the applied gradient is (1/W) * mean_r grad(L_r).  Every
loss term is a batch mean, so mean_r grad(L_r) over two 2-clip shards equals the gradient
of one process on the 4-clip batch: the DP gradient must be g_single / 2, and the DP
post-Adamax parameters those of Adamax applied to g_single / 2.

The ExtraTrainer case runs the num_pred_step=2 rollout: HRNet's backward runs twice into
one flat gradient, which must be all-reduced exactly once (GradSync.set_overlap)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H, W, B = 32, 64, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(n, frames):
    out = {}
    for i in range(n):
        g = torch.Generator().manual_seed(1000 + i)
        for k in range(1, frames + 1):
            out.setdefault(f"frame{k}", []).append(torch.rand((3, H, W), generator=g) * 2 - 1)
        for k in range(1, frames + 1):
            lab = torch.randint(0, 20, (H, W), generator=g)
            out.setdefault(f"seg{k}", []).append(torch.nn.functional.one_hot(lab, 20).permute(2, 0, 1).float())
    return {k: torch.stack(v) for k, v in out.items()}


def _trainer(kind, world, rank):
    from deep_video_interpolation_extrapolation_amd.options import default_args
    if kind == "inter":
        from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer as T
        args = default_args("INTER", syn_type="inter")
    else:
        from deep_video_interpolation_extrapolation_amd.runners.ExtraTrainer import ExtraTrainer as T
        args = default_args("EXTRA", syn_type="extra", num_pred_step=2)
    args.__dict__.update(train_coarse=True, batch_size=B, input_h=H, input_w=W, precision="fp32", synthetic=B,
                         num_workers=0, split="train", rank=rank, gpus=world)
    torch.manual_seed(1024)
    return T(args)


def _worker(rank, world, port, kind, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0", DVIE_PRECISION="fp32")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = _trainer(kind, world, rank)
        frames = 3 if kind == "inter" else 4
        data = _batch(B, frames)
        per = B // world
        mine = {k: v[rank * per:(rank + 1) * per] for k, v in data.items()}
        ld = tr.step(mine)
        hr = tr.model.module.coarse_model
        torch.cuda.synchronize()
        # numpy arrays travel by value (a shared tensor's fd would dangle once this process exits)
        q.put((rank, hr._flat_grad.cpu().numpy().copy(), hr._flat.detach().cpu().numpy().copy(), float(ld["loss_all"])))
    except BaseException as e:
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


def _dp_vs_single(dev, kind):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, g, flat, loss = q.get(timeout=400)
        res[r] = (g, flat, loss) if isinstance(g, str) else (torch.from_numpy(g), torch.from_numpy(flat), loss)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r][0], str), res[r][0]

    tr = _trainer(kind, 1, 0)
    hr = tr.model.module.coarse_model
    p0 = hr._flat.detach().cpu().clone()
    ld = tr.step(_batch(B, 3 if kind == "inter" else 4))
    torch.cuda.synchronize()
    g_single = hr._flat_grad.cpu().clone()

    g_dp, flat_dp, loss_dp = res[0]
    # every rank applied the same reduced gradient and holds the same parameters
    assert torch.equal(res[1][0], g_dp) and torch.equal(res[1][1], flat_dp)
    # logged loss: mean over ranks of the shard losses = the full-batch loss
    assert abs(loss_dp - float(ld["loss_all"])) <= 1e-4 * abs(float(ld["loss_all"]))
    want = g_single / world
    rel = float((g_dp - want).norm() / want.norm())
    tol = 1e-4 if kind == "inter" else 2e-3  # rollout: argmax one-hot of a prediction feeds step 2
    assert rel < tol, (kind, rel)
    # post-Adamax parameters = torch.optim.Adamax on g_single / W from the same start
    p = p0.clone().requires_grad_(True)
    p.grad = want.clone()
    torch.optim.Adamax([p], lr=tr.args.coarse_learning_rate).step()
    frac = float(((flat_dp - p.detach()).abs() > 1e-6).float().mean())
    assert frac < 1e-3, frac  # Adamax moves every weight by ~lr: only ~0 gradients may differ
    return rel


def _graph_worker(rank, world, port, q):
    """Eager trainer A: 3 steps; trainer B: 2 eager warm-up steps + capture + 1 replay, its
    gradient buckets all-reduced after the replayed graph segment that finishes them
    (GradSync.reduce_bucket).  Both on the same shard, W = 2."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0", DVIE_PRECISION="fp32",
                      DVIE_BUCKET_MB="4")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deep_video_interpolation_extrapolation_amd.runners.graph import GraphedStep
        data = _batch(B, 3)
        per = B // world
        mine = {k: v[rank * per:(rank + 1) * per].cuda() for k, v in data.items()}
        a = _trainer("inter", world, rank)
        la = [float(a.step(mine)["loss_all"]) for _ in range(3)]
        b = _trainer("inter", world, rank)
        gs = GraphedStep(b, mine, warmup=2)
        nev = len(gs.segments) - 1
        lb = float(gs.step()["loss_all"])
        torch.cuda.synchronize()
        ha, hb = a.model.module.coarse_model, b.model.module.coarse_model
        q.put((rank, (la, lb, nev) + tuple(t.detach().cpu().numpy().copy() for t in
                                           (ha._flat_grad, hb._flat_grad, ha._flat, hb._flat))))
    except BaseException as e:
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_graphed_dp2_step_overlaps_and_equals_eager(dev):
    """The captured W = 2 step (a graph segment per gradient bucket, each bucket's
    all-reduce issued behind its segment while the next ones replay) gives the eager W = 2
    step's gradients, parameters and logged loss."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_graph_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=500) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    res = {r: v[:3] + tuple(torch.from_numpy(a) for a in v[3:]) for r, v in res.items()}
    for r in range(world):
        la, lb, nev, ga, gb, fa, fb = res[r]
        assert nev >= 3, nev  # 39.7 MB of HRNet gradients in 4 MB buckets
        assert abs(lb - la[-1]) <= 1e-5 * abs(la[-1]), (la, lb)
        rel = float((gb - ga).norm() / ga.norm())
        assert rel < 1e-5, rel
        assert float((fb - fa).abs().max()) <= 1e-6, float((fb - fa).abs().max())
    assert torch.equal(res[0][4], res[1][4]) and torch.equal(res[0][6], res[1][6])


@pytest.mark.timeout(600)
def test_inter_step_dp2_equals_single_process(dev):
    _dp_vs_single(dev, "inter")


@pytest.mark.timeout(600)
def test_extra_rollout_dp2_reduces_once(dev):
    _dp_vs_single(dev, "extra")
