"""Plan compiler checks on CPU (descriptor lists are built; nothing is launched)."""
import os
import types

import numpy as np
import pytest
import torch

from deep_video_interpolation_extrapolation_amd import _lib as L
from deep_video_interpolation_extrapolation_amd import engine as E
from deep_video_interpolation_extrapolation_amd import nets

G = os.path.join(os.path.dirname(__file__), "golden")


def make(**kw):
    a = types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet")
    a.__dict__.update(kw)
    torch.manual_seed(1024)
    return nets.InterNet(a)


def test_param_names_and_seeded_init_match_reference():
    f = np.load(os.path.join(G, "hrnet_fwd.npz"))
    m = make()
    sd = m.coarse_model.state_dict()
    names = [str(n) for n in f["param_names"]]
    assert sorted(sd) == names
    cs = np.array([[float(sd[n].double().sum()), float((sd[n].double() ** 2).sum())] for n in names])
    np.testing.assert_allclose(cs, f["param_checksums"], rtol=1e-12, atol=1e-12)
    assert sum(p.numel() for p in m.parameters()) == int(f["n_params"])


def test_params_are_views_of_one_flat_buffer():
    hr = make().coarse_model
    base = hr._flat.data_ptr()
    end = base + hr._flat.numel() * 4
    for p in hr.parameters():
        assert base <= p.data_ptr() < end


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_hrnet_plan_structure(dtype, fused, monkeypatch):
    """77 reference convs; with the two 1x1 head convs stacked into one 448 -> 896 conv
    (E.StackedConv, the default) the plan has 76, and the stacked output's two halves --
    read by rgb_layer.2 and seg_layer.2 -- each receive their gradient."""
    from deep_video_interpolation_extrapolation_amd.nets.HRNet import HRNet
    monkeypatch.setattr(HRNet, "fuse_heads", fused)
    hr = make().coarse_model
    g = hr._lower(E.Graph(dtype), 32, 64)
    plan = g.compile(2, torch.device("cpu"), backward=True)
    kinds = plan.describe()["kinds"]
    n_conv_fwd = sum(1 for op in g.ops if isinstance(op, E.ConvOp))
    n_ref = 76 if fused else 77
    assert n_conv_fwd == n_ref
    heads = [b for b in g.buffers if b.name == "heads_hidden"]
    assert len(heads) == int(fused)
    if fused:
        assert sorted(heads[0].expected) == [(0, 448), (448, 448)] and heads[0].dact_done
    # every trainable conv gets one wgrad; stride-2 dgrads split into 4 phases; in bf16 the
    # rgb output head's data + weight gradients are one fused launch (dvie_head3_bwd; the seg
    # head stays unfused by default, DVIE_HEAD3_FUSED) and each frame's segmentation encoder
    # runs its backward -- three weight gradients and two data gradients -- as one
    # dvie_segenc_bwd launch, and its forward -- three convs -- as one dvie_segenc_fwd launch
    # (DVIE_SEGENC_FWD=0: three)
    n_head3 = 1 if dtype == torch.bfloat16 else 0
    n_seg = 2 if dtype == torch.bfloat16 else 0
    assert kinds.get(L.OP_HEAD3_BWD, 0) == n_head3
    assert kinds.get(L.OP_SEGENC_FWD, 0) == n_seg and kinds.get(L.OP_SEGENC_BWD, 0) == n_seg
    assert kinds[L.OP_WGRAD] == n_ref - n_head3 - 3 * n_seg
    n_s2 = sum(1 for op in g.ops if isinstance(op, E.ConvOp) and op.layer.stride == 2)
    n_dgrad = sum(1 for op in g.ops if isinstance(op, E.ConvOp) and op.x.buf.needs_grad)
    # bf16: the stride-2 data gradients with <= 128 input channels run as ONE phase-split
    # launch (dvie_conv_desc.phc) instead of four
    n_ph4 = sum(1 for o in plan.bwd if o.kind == L.OP_CONV and o.u.conv.phc)
    n_ph4_want = sum(1 for op in g.ops if isinstance(op, E.ConvOp) and op.layer.stride == 2 and op.x.buf.needs_grad
                     and op.layer.cin_p <= 128) if dtype == torch.bfloat16 else 0
    assert n_ph4 == n_ph4_want
    assert kinds[L.OP_CONV] == n_conv_fwd + n_dgrad + 3 * (n_s2 - n_ph4) - n_head3 - 2 * n_seg - 3 * n_seg
    # every buffer that needs a gradient received all of its contributions
    for b in g.buffers:
        if b.needs_grad and b.expected:
            assert b.done


@pytest.mark.parametrize("dtype,stacked", [(torch.float32, False), (torch.bfloat16, True)])
def test_stacked_heads_fit_the_buffer_range(dtype, stacked):
    """At 1024x2048 the stacked 896-channel hidden map is 7.5 GB per image in fp32, past
    the 32-bit buffer range the 3x3 output convs address one image through: the heads
    stay separate there (bf16: 3.8 GB, stacked)."""
    hr = make().coarse_model
    g = hr._lower(E.Graph(dtype), 1024, 2048)
    assert any(b.name == "heads_hidden" for b in g.buffers) == stacked


def test_highres_large_builds():
    hr = make(highres_large=True).coarse_model
    g = hr._lower(E.Graph(torch.float32), 32, 64)
    plan = g.compile(1, torch.device("cpu"), backward=True)
    assert plan.describe()["n_bwd"] > 0


def test_vgg_plan_structure():
    from deep_video_interpolation_extrapolation_amd.nets.vgg import my_vgg, vgg19_features
    v = my_vgg(vgg19_features())
    g = E.Graph(torch.float32)
    v.lower(g, 32, 64, normalize=True, loss=True)
    plan = g.compile(4, torch.device("cpu"), n_bwd=2, backward=True)
    k = plan.describe()["kinds"]
    assert L.OP_WGRAD not in k  # frozen
    assert g.n_l1 == 5


def test_vgg_synthetic_weights_match_oracle():
    from deep_video_interpolation_extrapolation_amd.nets.vgg import synthetic_vgg19_state as a
    from oracle.losses import synthetic_vgg19_state as b
    sa, sb = a(), b()
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k])


@pytest.mark.parametrize("bucket_mb", [0.25, 4, 16])
def test_buckets_with_unstacked_heads(bucket_mb, monkeypatch):
    """The flat parameter layout comes from a dry lowering with the two 1x1 head convs
    stacked; a plan that keeps them separate (fp32 at 1024x2048: the stacked hidden map
    passes the 32-bit buffer range) completes rgb_layer.0 and seg_layer.0 one by one.  The
    in-backward all-reduce buckets must still tile the flat buffer, and every parameter of a
    bucket must have completed at its cut (here: the stacking limit forced to 0 after
    construction, at 32x64)."""
    from deep_video_interpolation_extrapolation_amd.nets.HRNet import HRNet
    hr = make().coarse_model
    monkeypatch.setattr(HRNet, "_stack_limit", 0)
    g = hr._lower(E.Graph(torch.float32), 32, 64)
    assert not any(b.name == "heads_hidden" for b in g.buffers)
    assert any(lay.name == "rgb_layer.0" for lay in g.layers)
    plan = g.compile(1, torch.device("cpu"), backward=True)
    cuts, ranges = hr._buckets(plan, int(bucket_mb * 2 ** 20))
    total = hr._flat.numel()
    assert ranges[0][0] == 0 and ranges[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert len(cuts) == len(ranges) - 1
    # at each cut every parameter below the range end has completed
    span = {id(p): (off, off + n) for p, (off, n, _) in zip(hr._flat_params, hr._flat_specs)}
    # (several layers complete at one index when their reductions share a batched launch:
    # a cut is checked once every completion at its index is counted)
    done = []
    k = 0
    comps = plan.completions
    for j, (idx, lay) in enumerate(comps):
        ps = lay.m.params() if isinstance(lay.m, E.StackedConv) else [lay.m.weight] + (
            [lay.m.bias] if lay.m.bias is not None else [])
        done += [span[id(p)] for p in ps]
        last_at_idx = j + 1 == len(comps) or comps[j + 1][0] != idx
        while last_at_idx and k < len(cuts) and idx == cuts[k]:
            hi = ranges[k][1]
            assert sum(e - s for s, e in done if e <= hi) == hi
            k += 1
    assert k == len(cuts)
    if bucket_mb <= 4:
        assert len(cuts) >= 2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_weight_lane_tags(dtype, monkeypatch):
    """Executor lanes of a compiled HRNet plan (include/dvie.h dvie_op.lane): every weight /
    bias gradient op (WGRAD, WREDUCE, COLSUM) is on the weight lane 1 and every other op, in
    both directions, on the caller's stream (lane 0); DVIE_WGRAD_LANE=0 puts everything on
    lane 0."""
    for env, wl in (("1", 1), ("0", 0)):
        monkeypatch.setenv("DVIE_WGRAD_LANE", env)
        hr = make().coarse_model
        g = hr._lower(E.Graph(dtype), 32, 64)
        plan = g.compile(2, torch.device("cpu"), backward=True)
        n_w = 0
        for i in range(plan.n_bwd):
            o = plan.bwd_arr[i]
            if o.kind in (L.OP_WGRAD, L.OP_WREDUCE, L.OP_COLSUM, L.OP_WREDUCE_MULTI):
                assert o.lane == wl
                n_w += 1
            else:
                assert o.lane == 0, o.kind
        assert n_w > 40
        assert all(plan.fwd_arr[i].lane == 0 for i in range(len(plan.fwd_arr)))


def test_batched_reductions(monkeypatch):
    """The weight lane's slab reductions run in batches (engine Plan._batch_reductions): no
    one-by-one reduction left, at most 16 per batch, every parameter's gradient slot points
    into a batch, the completion points stay ordered and after their batch, and the slab
    regions of one batch do not overlap (each writer its own, the stride-2 phase launches of
    one layer one shared region)."""
    hr = make().coarse_model
    g = hr._lower(E.Graph(torch.bfloat16), 32, 256)
    plan = g.compile(2, torch.device("cpu"), backward=True)
    kinds = [plan.bwd_arr[i].kind for i in range(plan.n_bwd)]
    assert L.OP_WREDUCE not in kinds and kinds.count(L.OP_WREDUCE_MULTI) >= 5
    n_red = 0
    for i, k in enumerate(kinds):
        if k == L.OP_WREDUCE_MULTI:
            m = plan.bwd_arr[i].u.wreduce_multi
            assert 1 <= m.n <= 16
            n_red += m.n
    assert n_red == sum(1 for s in plan._grad_slots if s[2] != "bn")
    for idx, lay, which, first in plan._grad_slots:
        assert isinstance(idx, tuple) and kinds[idx[1]] == L.OP_WREDUCE_MULTI
    comp = [c for c, _ in plan.completions]
    assert comp == sorted(comp) and all(kinds[c - 1] == L.OP_WREDUCE_MULTI for c in comp)
    # the slab ranges the reductions of one batch read from the shared workspace are disjoint
    ws0, ws1 = plan.ws.data_ptr(), plan.ws.data_ptr() + 4 * plan.ws.numel()
    for i, k in enumerate(kinds):
        if k != L.OP_WREDUCE_MULTI:
            continue
        m = plan.bwd_arr[i].u.wreduce_multi
        descs = (L.WreduceDesc * m.n).from_address(m.descs)
        rs = sorted((d.ws, d.ws + 4 * d.splits * d.ws_rows * d.ws_k) for d in descs if ws0 <= d.ws < ws1)
        assert all(a[1] <= b[0] for a, b in zip(rs, rs[1:])), rs
        assert all(e <= ws1 for _, e in rs)


def test_fused_segenc_backward_leaves_no_dead_work():
    """bf16 HRNet plan with the fused segmentation-encoder backward (dvie_segenc_bwd): the
    encoder's hidden maps e1 / e2 get no gradient storage (d_e1 / d_e2 stay on chip in that
    kernel), and no backward op applies an ELU derivative to a gradient nobody reads (the
    r04 plan emitted one such EW_COPY per map and frame)."""
    hr = make().coarse_model
    g = hr._lower(E.Graph(torch.bfloat16), 32, 64)
    plan = g.compile(2, torch.device("cpu"), backward=True)
    assert plan.describe()["kinds"].get(L.OP_SEGENC_BWD, 0) == 2
    inner = [b for b in g.buffers if b.name.startswith("seg") and b.name.endswith(("_e1", "_e2"))]
    assert len(inner) == 4 and all(b.g is None for b in inner)
    for i in range(plan.n_bwd):
        o = plan.bwd_arr[i]
        if o.kind == L.OP_EW:
            assert o.u.ew.dact != L.ACT_ELU, "an ELU derivative pass is left in the backward"


def test_pack_blocks_from_the_library():
    """The flat pack grid's per-descriptor block counts come from the library
    (dvie_pack_blocks), and the descriptors' blk0 tile the grid."""
    hr = make().coarse_model
    g = hr._lower(E.Graph(torch.bfloat16), 32, 64)
    plan = g.compile(2, torch.device("cpu"), backward=True)
    descs = plan._pack_descs
    blk = 0
    for d in descs:
        assert d.blk0 == blk
        blk += L.load().dvie_pack_blocks(__import__("ctypes").byref(d))
    assert plan.fwd_arr[0].u.pack.blocks == blk
