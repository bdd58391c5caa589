"""Data-parallel host logic at world_size 2 over gloo on CPU (no GPU, nothing launched).

Covers what runners/comm.py and the trainers do across ranks:
  * DDP-style initial parameter broadcast (GradSync.__init__);
  * the in-backward gradient buckets: ranges cover the flat gradient buffer exactly, in
    backward-completion order, and the per-bucket SUM all-reduces produce the sum over
    ranks of every gradient element;
  * the coalesced loss sync (one all_reduce for all logged scalars, mean over ranks);
  * the DistributedSampler-style shard: disjoint, together the whole dataset, per-rank
    batch = bs // W (reference runners/InterTrainer.py:84-87).
"""
import os
import socket
import types

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from collections import OrderedDict

        from deep_video_interpolation_extrapolation_amd import engine as E
        from deep_video_interpolation_extrapolation_amd import nets
        from deep_video_interpolation_extrapolation_amd.data import SyntheticClips
        from deep_video_interpolation_extrapolation_amd.runners import comm

        # different init per rank: the broadcast must make rank 1 equal rank 0
        torch.manual_seed(1024 + rank)
        a = types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet")
        model = nets.InterNet(a)
        hr = model.coarse_model
        sync = comm.GradSync(model, bucket_mb=4)
        assert sync.W == world
        ref = hr._flat.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(hr._flat, ref), "parameter broadcast"

        # bucket ranges of a compiled (CPU, descriptor-only) training plan
        g = hr._lower(E.Graph(torch.float32), 16, 32)
        plan = g.compile(2, torch.device("cpu"), backward=True)
        cuts, ranges = hr._buckets(plan, sync.bucket_bytes)
        assert ranges[0][0] == 0 and ranges[-1][1] == hr._flat.numel()
        assert all(r0[1] == r1[0] for r0, r1 in zip(ranges, ranges[1:]))
        assert cuts == sorted(cuts) and len(cuts) == len(ranges) - 1
        assert len(ranges) > 2  # 39.7 MB of gradients in 4 MB buckets

        fg = hr.flat_grad()
        gen = torch.Generator().manual_seed(77 + rank)
        fg.copy_(torch.randn(fg.shape, generator=gen))
        mine = fg.clone()
        hook = hr.grad_hook[1]
        for lo, hi in ranges:  # as run_backward calls it, one bucket per cut
            hook(lo, hi)
        sync.wait()
        tot = mine.clone()
        dist.all_reduce(tot)
        assert torch.allclose(fg, tot, rtol=0, atol=1e-6), "bucketed all-reduce"

        # graph-capture mode (runners/graph.py): the hooks hand each finished bucket to the
        # capture's segment cut in bucket order and launch nothing; the replay issues one
        # all-reduce per bucket, in the same order on every rank, then the rest
        fg.copy_(torch.randn(fg.shape, generator=gen))
        mine = fg.clone()
        cutlist = []
        sync.capture_cut = lambda owner, lo, hi: cutlist.append((owner, lo, hi))
        for lo, hi in ranges:
            hook(lo, hi)
        sync.capture_cut = None
        assert [(lo, hi) for _, lo, hi in cutlist] == ranges and not sync.works
        order = torch.tensor([x for _, lo, hi in cutlist for x in (lo, hi)])
        orders = [torch.zeros_like(order) for _ in range(world)]
        dist.all_gather(orders, order)
        assert all(torch.equal(o, orders[0]) for o in orders), "bucket order differs across ranks"
        assert torch.equal(fg, mine), "capture mode launched a collective"
        for bucket in cutlist:
            sync.reduce_bucket(*bucket)
        sync.reduce_rest(True)
        tot = mine.clone()
        dist.all_reduce(tot)
        assert torch.allclose(fg, tot, rtol=0, atol=1e-6), "replayed bucket all-reduce"

        ld = OrderedDict(a=torch.tensor(float(rank)), b=torch.tensor(2.0 * rank + 1))
        out = comm.sync_losses(ld, world)
        assert abs(float(out["a"]) - 0.5) < 1e-7 and abs(float(out["b"]) - 2.0) < 1e-7

        ds = SyntheticClips(10, 8, 16)
        sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True,
                                                                  seed=1024)
        idx = torch.tensor(list(iter(sampler)))
        allidx = [torch.zeros_like(idx) for _ in range(world)]
        dist.all_gather(allidx, idx)
        cat = torch.cat(allidx)
        assert sorted(set(cat.tolist())) == list(range(10)) and len(cat) == 10
        q.put((rank, "ok"))
    except BaseException as e:  # report to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
