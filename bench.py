"""Throughput benchmark: InterNet (HRNet) training steps on synthetic 256x512 len-3 clips.

    python bench.py [--gpus N --steps K --warmup W]            (N>1: launched by torchrun)

Workload (BASELINE.json configs[1]): InterNet int_5_len_3, 256x512, bf16 compute, per-GPU
batch 8 synthetic Cityscapes-shaped triplets resident in HBM; one step = the reference's
InterTrainer step body (HRNet fwd, RGBLoss (L1+GDL+SSIM+VGG19) + 30*CE, backward, RCCL
gradient all-reduce, Adamax).  Metric: synthesized frames/s (one per clip), whole job.

After the timed region, 2 extra profiling steps time every plan op with HIP events on the
launch stream; the dominant kernel family (the conv forward + data-gradient kernels) is
reported against the bf16 MFMA peak as `roofline`.  Rank 0 at N=1 also times the
CPU oracle (the reference algorithm restated in PyTorch-CPU fp32) on a bounded sample as
`cpu_baseline`.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0  # dense MFMA (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0
KIND_NAMES = {2: "conv_wgrad", 3: "wgrad_reduce", 4: "bias_colsum", 5: "pointwise", 6: "loss", 7: "weight_pack",
              8: "batchnorm_fwd", 9: "batchnorm_bwd", 10: "head_fwd", 11: "head_bwd"}
# HBM bytes per launch of the conv fwd+dgrad family from PMC counters (tools/pmc_bench.sh on
# this same bench command; FETCH_SIZE x2 gfx950 correction), committed under profiles/
# per workload; None: no PMC pass on this workload -> "traffic": null
PMC_DIRS = {"c2": "r06final/pmc", "c5": None}



class _StderrLog:
    def info(self, msg):
        print(msg, file=sys.stderr, flush=True)

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (clips); default: the workload's")
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=2)
    ap.add_argument("--ops-out", default=None, help="write the per-op profile table (profiling steps) here")
    ap.add_argument("--workload", default="c2", choices=["c2", "c5"],
                    help="c2: BASELINE configs[1] (InterNet 256x512 bf16, batch 8; the default line); c5: "
                         "BASELINE configs[4] per GPU (two-stage extrapolation ExtraStage3Net 1024x2048 bf16, batch "
                         "1, hipGraph-captured step)")
    ap.add_argument("--graph", type=int, default=None,
                    help="1: time the hipGraph-captured step (runners/graph.py), 0: the eager step; default 0 for "
                         "c2 (same box, r04v: eager 34.9 ms with the executor's weight lane vs 35.4 ms captured -- "
                         "a capture keeps every op on one stream), 1 for c5 (the config names a captured step)")
    return ap.parse_args()


def make_batch(n, H, W, device, first):
    from deep_video_interpolation_extrapolation_amd.data import SyntheticClips
    ds = SyntheticClips(first + n, H, W, 3)
    items = [ds[first + i] for i in range(n)]
    return {k: torch.stack([it[k] for it in items]).to(device) for k in items[0]}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(H, W, steps=2):
    """CPU oracle InterTrainer steps (the reference algorithm restated in PyTorch-CPU fp32)
    on bounded samples, BASELINE.md's CPU plan: one untimed warm-up step, then
    * the bench workload's frame size (H x W, batch 2): `steps` timed steps -> value;
    * C1 (8 triplets at 128x256, batch 2 = 4 steps), timed whole -> c1_frames_per_s."""
    from oracle import hrnet, losses, step
    threads = torch.get_num_threads()
    P = hrnet.init_params(1024)
    vs = losses.synthetic_vgg19_state()
    step.inter_step(P, vs, step.synthetic_batch(2, 64, 128))  # warm-up (untimed)
    B = 2
    t = time.time()
    for k in range(steps):
        step.inter_step(P, vs, step.synthetic_batch(B, H, W, first_index=B * k))
    dt = time.time() - t
    t1 = time.time()
    for k in range(4):
        step.inter_step(P, vs, step.synthetic_batch(2, 128, 256, first_index=2 * k))
    dt1 = time.time() - t1
    return {"value": B * steps / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "os_cpu_count": os.cpu_count(), "torch_threads": threads, "cpu_model": _cpu_model(),
            "c1_frames_per_s": round(8 / dt1, 4),
            "sample": f"{steps} InterTrainer steps of the CPU oracle (fp32) at {H}x{W}, batch {B} ({dt:.1f}s), after "
                      f"one untimed warm-up step; C1: 8 triplets at 128x256 in 4 steps of batch 2 ({dt1:.1f}s)"}


def cpu_baseline_c5(H=256, W=512):
    """CPU oracle two-stage extrapolation step (oracle.step.extra_refine_step, fp32) on a
    bounded sample: one step of batch 1 at H x W (a 1024x2048 step takes minutes on the
    host), after an untimed warm-up step at 64x128; `value` is that sample's frames/s and
    `per_pixel_scaled` the same rate scaled to 1024x2048 frames by pixel count."""
    from oracle import hrnet, losses, refine, step
    threads = torch.get_num_threads()
    Pc, vs = hrnet.init_params(1024), losses.synthetic_vgg19_state()
    Pr, Ps = refine.init_params(None, refine.srn_specs()), refine.init_params(None, refine.attn_specs())
    step.extra_refine_step(Pc, Pr, vs, step.synthetic_batch(1, 64, 128), 3, Ps=Ps, prop=True)
    t = time.time()
    step.extra_refine_step(Pc, Pr, vs, step.synthetic_batch(1, H, W), 3, Ps=Ps, prop=True)
    dt = time.time() - t
    return {"value": round(1 / dt, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "per_pixel_scaled": round(1 / dt * (H * W) / (1024 * 2048), 5), "os_cpu_count": os.cpu_count(),
            "cpu_model": _cpu_model(),
            "sample": f"1 two-stage extrapolation step of the CPU oracle (fp32, n_sc 3, stage3_prop) at {H}x{W}, "
                      f"batch 1 ({dt:.1f}s), after one untimed warm-up step at 64x128"}


def warp_roofline(dev, n, H, W, reps=20):
    """The optical-flow warp (FlowWrapper, utils/net_utils.py:89-114; dormant in the
    InterNet step) on (n, 3, H, W) frames: dvie_warp_fwd / dvie_warp_bwd launched back to back
    through the C ABI (no autograd or allocation between launches), timed with HIP events on
    the launch stream, against the HBM roofline.  Algorithmic bytes per pixel (fp32):
    forward img 12 + flow 8 + out 12 = 32; backward img 12 + flow 8 + dout 12 + dimg 12 +
    dflow 8 = 52 (dimg is overwritten: no zero-fill)."""
    import ctypes
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.rand((n, 3, H, W), generator=g, device=dev)
    # smooth optical-flow-like field: up to ~4 px at 256x512 (the same normalised field at
    # other sizes) plus 0.1 px noise; per-pixel random flow is a gather/scatter stress test,
    # not optical flow
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H, device=dev), torch.linspace(0, 1, W, device=dev), indexing="ij")
    flow = torch.stack([torch.sin(6.3 * xx + 3.1 * yy) * 0.016, torch.cos(4.7 * yy - 2.9 * xx) * 0.024])
    flow = flow.unsqueeze(0).repeat(n, 1, 1, 1) + (torch.rand((n, 2, H, W), generator=g, device=dev) - 0.5) * 4e-4
    go = torch.randn((n, 3, H, W), generator=g, device=dev)
    out, dx, dflow = torch.empty_like(x), torch.zeros_like(x), torch.empty_like(flow)
    d = L.WarpDesc()
    d.img, d.flow, d.out, d.dout, d.dimg, d.dflow = (t.data_ptr() for t in (x, flow, out, go, dx, dflow))
    d.n, d.c, d.h, d.w, d.align_corners = n, 3, H, W, 1
    ws = torch.empty(lib.dvie_warp_ws_floats(ctypes.byref(d)), device=dev)
    d.ws = ws.data_ptr()
    s = L.stream_ptr(dev)

    def fwd():
        L.check(lib.dvie_warp_fwd(ctypes.byref(d), L.stream_ptr(dev)), "warp fwd")

    def bwd():
        L.check(lib.dvie_warp_bwd(ctypes.byref(d), L.stream_ptr(dev)), "warp bwd")

    # The launches are timed two ways: replayed from a captured hipGraph of `reps` launches
    # (the GPU time per launch: at 256x512 a launch is ~7 us, about what the Python ctypes
    # call + hipLaunchKernel take, so eager back-to-back launches leave the GPU idle between
    # kernels), which gives `*_ms` / `*_frac`; and eagerly from Python (`*_ms_eager`).
    def floor():  # an empty kernel on the forward's grid (dvie_warp_fwd: 4 waves per block)
        waves = n * H * ((W + 255) // 256)
        L.check(lib.dvie_launch_probe(min((waves + 3) // 4, 8192), 256, L.stream_ptr(dev)), "launch probe")

    res = {}
    for tag, fn, bpp in (("fwd", fwd, 32.0), ("bwd", bwd, 52.0), ("floor", floor, 0.0)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms_eager = e0.elapsed_time(e1) / reps
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        del g
        if tag == "floor":  # the forward's launch floor: an empty kernel of its grid
            res["fwd_launch_floor_ms"] = round(ms, 4)
            res["fwd_frac_above_floor"] = round(32.0 * n * H * W / ((res["fwd_ms"] - ms) * 1e-3) / 1e9 / PEAK_HBM_GBS, 4) \
                if res["fwd_ms"] > ms else None
            continue
        gbs = bpp * n * H * W / (ms * 1e-3) / 1e9
        res[tag + "_ms"], res[tag + "_GBps"], res[tag + "_frac"] = round(ms, 4), round(gbs, 1), round(gbs / PEAK_HBM_GBS, 4)
        res[tag + "_ms_eager"] = round(ms_eager, 4)
        res[tag + "_frac_eager"] = round(bpp * n * H * W / (ms_eager * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
    res.update(shape=[n, 3, H, W], bytes_per_px={"fwd": 32, "bwd": 52}, timing="hipGraph replay of back-to-back launches",
               flow="smooth, |dx| <= %.1f px, |dy| <= %.1f px" % (0.016 * (W - 1) / 2, 0.024 * (H - 1) / 2))
    return res


def mfma_probe(dev, blocks=2048, iters=16384, reps=5):
    """Dense bf16 MFMA rate this box sustains under load (dvie_mfma_probe: 4-wave workgroups filling every CU,
    back-to-back v_mfma_f32_32x32x16_bf16 on pseudo-random register operands, 32768 FLOP
    each), timed with HIP events on the launch stream.  The chip lowers its clock under
    random-data MFMA load (MI355X_MICROARCH.md), so this, not the 2.5 PF spec, is the ceiling
    a conv kernel can reach on the same box; reported beside `frac` as `frac_of_mfma_loop`."""
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    out = torch.empty(blocks * 256, device=dev)
    s = L.stream_ptr(dev)
    for _ in range(10):  # ~0.3 s of load first, so the clock has settled
        L.check(lib.dvie_mfma_probe(out.data_ptr(), blocks, iters, s), "mfma probe")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        L.check(lib.dvie_mfma_probe(out.data_ptr(), blocks, iters, s), "mfma probe")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flop = blocks * 4 * 8 * iters * 32768.0
    return {"tflops": round(flop / (ms * 1e-3) / 1e12, 1), "ms": round(ms, 3), "blocks": blocks, "iters": iters,
            "finite": bool(torch.isfinite(out).all())}


def clip_prep_roofline(dev, n, H, W, reps=20):
    """Device clip pipeline (data.DeviceClips / dvie_clip_prep; the reference's DataLoader
    worker, folder.py:207-247): n 3-frame clips from an HBM-resident uint8 store of
    (H+22)x(W+22) frames, flipped + pseudo-motion cropped to HxW, normalised, 20-class
    one-hot.  Algorithmic bytes per output pixel: read RGB 3 + label 1, write 12 + 80 = 96."""
    import random
    import numpy as np
    from deep_video_interpolation_extrapolation_amd.data import DeviceClips
    g = torch.Generator(device=dev).manual_seed(3)
    h0, w0 = H + 22, W + 22
    imgs = torch.randint(0, 256, (n, 3, h0, w0, 3), generator=g, device=dev, dtype=torch.uint8)
    segs = torch.randint(0, 20, (n, 3, h0, w0), generator=g, device=dev, dtype=torch.uint8)
    dc = DeviceClips(imgs, segs, crop=(H, W), device=dev, strict=False)
    params = dc.draw_params(n, np.random.RandomState(0), random.Random(0))
    idx = list(range(n))
    for _ in range(3):
        dc.batch(idx, params)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        dc.batch(idx, params)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = 96.0 * n * 3 * H * W / (ms * 1e-3) / 1e9
    return {"clips": n, "frames": 3 * n, "shape": [H, W], "ms": round(ms, 4), "GBps": round(gbs, 1),
            "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_px": 96,
            "note": "per batch call incl. its small host->device index/param copies and output allocation"}


def launch_command(a, argv, port):
    """`bench.py --gpus N` (N > 1) started as a plain process: the torchrun command that
    runs it as N ranks, one per GPU (the reference's one-process-per-GPU launch,
    main.py:133-154, which mp.spawn's `gpus` workers)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# per-GPU batch and frame size of each workload (BASELINE.json configs[1] / configs[4])
WORKLOAD_SHAPE = {"c2": dict(batch=8, height=256, width=512), "c5": dict(batch=1, height=1024, width=2048)}


def refuse_timing_switches(env=os.environ):
    """Timing-only ablation switches (DVIE_*_DBG) skip stores, MFMAs or operand streams in the
    kernels of a -DDVIE_TIMING_DBG build; a bench line must never run with one set."""
    bad = sorted(k for k in env if k.startswith("DVIE_") and k.endswith("_DBG") and env[k] not in ("", "0"))
    if bad:
        print(f"bench.py: refusing to run with timing-only switches set: {', '.join(bad)}", file=sys.stderr)
        sys.exit(2)


def main():
    refuse_timing_switches()
    a = parse()
    if a.graph is None:
        a.graph = 1 if a.workload == "c5" else 0
    for k, v in WORKLOAD_SHAPE[a.workload].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # nothing has touched the GPU yet: run the N ranks as a child torchrun and exit with
        # its status (never exec from here)
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(launch_command(a, sys.argv[1:], _free_port()), env=env))
    os.environ["DVIE_PRECISION"] = a.precision
    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert world == a.gpus or a.gpus == 1, f"--gpus {a.gpus} but WORLD_SIZE={world}"
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from deep_video_interpolation_extrapolation_amd import engine
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer

    common = dict(mode="xs2xs", vid_length=1, train_coarse=True, batch_size=a.batch * world, input_h=a.height,
                  input_w=a.width, precision=a.precision, synthetic=a.batch * world, num_workers=0, split="train",
                  rank=rank, gpus=world)
    if a.workload == "c5":
        from deep_video_interpolation_extrapolation_amd.runners.ExtraTrainer import ExtraTrainer
        # the reference's own two-stage command line (cmd:158): --n_sc 3 --stage3 --stage3_prop,
        # here with all three nets trained
        args = default_args("EXTRA", syn_type="extra", interval=9, model="ExtraStage3Net", refine=True,
                            refine_model="SRNRefine", stage3=True, stage3_prop=True, n_scales=3, train_refine=True,
                            train_stage3=True, **common)
        trainer_cls = ExtraTrainer
    else:
        args = default_args("INTER", syn_type="inter", interval=5, **common)
        trainer_cls = InterTrainer
    args.logger = _StderrLog()  # stdout carries the one JSON line only
    torch.manual_seed(args.seed)
    trainer = trainer_cls(args)
    data = make_batch(a.batch, a.height, a.width, dev, rank * a.batch)

    def timed(fn):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            out = fn(data)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t)
        return dt, out

    for _ in range(a.warmup):
        trainer.step(data)
    eager_dt, ld = timed(trainer.step)
    dt = eager_dt
    if a.graph:
        from deep_video_interpolation_extrapolation_amd.runners.graph import GraphedStep
        gstep = GraphedStep(trainer, data, warmup=1)  # the batch now lives in the graph's static inputs
        dt, ld = timed(lambda _d: gstep.step())
        loss_all = float(ld["loss_all"])
        gstep.close()  # eager profiling steps below: in-backward bucket overlap back on (W > 1)
    else:
        loss_all = float(ld["loss_all"])

    # ---- profiling steps: per-op HIP events on the launch stream ----
    prof = []
    if a.profile_steps > 0:
        engine.PROFILE = prof
        for _ in range(a.profile_steps):
            trainer.step(data)
        torch.cuda.synchronize()
        engine.PROFILE = None
    agg = {}
    per_op = {}
    roof_t = {}  # per-op roofline time: max(F / P_mfma, B / BW_hbm)
    peak = PEAK_BF16_TFLOPS if a.precision == "bf16" else PEAK_FP32_TFLOPS
    for meta, kind, e0, e1 in prof:
        ms = e0.elapsed_time(e1)
        cls = meta["cls"] if meta else KIND_NAMES.get(kind, f"kind{kind}")
        r = agg.setdefault(cls, dict(ms=0.0, n=0, flops=0.0, bytes=0.0, roof_ms=0.0))
        r["ms"] += ms
        r["n"] += 1
        if meta:
            f, b = meta.get("flops", 0.0), meta.get("bytes", 0.0)
            r["flops"] += f
            r["bytes"] += b
            r["roof_ms"] += 1e3 * max(f / (peak * 1e12), b / (PEAK_HBM_GBS * 1e9))
            o = per_op.setdefault((cls, meta.get("name", "?")), dict(ms=0.0, n=0, flops=0.0, bytes=0.0))
            o["ms"] += ms
            o["n"] += 1
            o["flops"] += f
            o["bytes"] += b
    conv = [agg[c] for c in ("conv_fwd", "conv_dgrad") if c in agg]
    roof = None
    if conv:
        ms = sum(r["ms"] for r in conv)
        n = sum(r["n"] for r in conv)
        fl = sum(r["flops"] for r in conv)
        by = sum(r["bytes"] for r in conv)
        tf = fl / (ms * 1e-3) / 1e12
        traffic = wg_traffic = None
        pmc_dir = PMC_DIRS.get(a.workload)
        pmc_file = os.path.join(ROOT, "profiles", pmc_dir, "traffic.json") if pmc_dir else None
        if pmc_file and os.path.exists(pmc_file):
            pm = json.load(open(pmc_file))
            t, tw = pm.get("conv"), pm.get("wgrad")
            traffic = round(t["bytes_per_launch"]) if t else None
            wg_traffic = round(tw["bytes_per_launch"]) if tw else None
        roof = {"bound": "mfma", "achieved": round(tf, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(tf / peak, 4),
                "traffic": traffic, "traffic_unit": "HBM bytes/launch (PMC FETCH_SIZEx2 + WRITE_SIZE, "
                                                     f"profiles/{pmc_dir})" if traffic is not None else None,
                "algorithmic_bytes_per_launch": round(by / max(1, n)),
                "kernel": "conv fwd+dgrad family (conv_h8 / conv_halo / conv_strip / conv_narrow / conv_nk / conv1x1 / "
                          "conv1x1_ring / conv_s2 / conv_igemm / head3_bwd / segenc_fwd kernels)",
                "launches_per_step": n // max(1, a.profile_steps),
                "avg_launch_us": round(ms * 1e3 / max(1, n), 2),
                "algorithmic_tflop_per_step": round(fl / a.profile_steps / 1e12, 4),
                # sum over launches of max(F/P_mfma, B/BW_hbm) over measured time
                "per_op_roofline_time_frac": round(sum(r["roof_ms"] for r in conv) / ms, 4)}
        mp = mfma_probe(dev) if a.precision == "bf16" else None
        if mp:
            roof["mfma_loop"] = mp
            roof["frac_of_mfma_loop"] = round(tf / mp["tflops"], 4)
        wg = agg.get("conv_wgrad")
        if wg:  # weight gradients: algorithmic bytes (x, dy read once, dW written) vs PMC traffic
            roof["wgrad"] = {"launches_per_step": wg["n"] // max(1, a.profile_steps),
                             "avg_launch_us": round(wg["ms"] * 1e3 / max(1, wg["n"]), 2),
                             "tflops": round(wg["flops"] / (wg["ms"] * 1e-3) / 1e12, 2),
                             "algorithmic_bytes_per_launch": round(wg["bytes"] / max(1, wg["n"])),
                             "traffic": wg_traffic}
    if a.ops_out and rank == 0:
        with open(a.ops_out, "w") as f:
            f.write(f"{'class':12s} {'layer':42s} {'n':>3s} {'ms':>8s} {'TFLOP/s':>8s} {'GB/s':>8s} {'roof%':>6s}\n")
            for (cls, name), o in sorted(per_op.items(), key=lambda kv: -kv[1]["ms"]):
                t = o["ms"] * 1e-3
                rt = max(o["flops"] / (peak * 1e12), o["bytes"] / (PEAK_HBM_GBS * 1e9))
                f.write(f"{cls:12s} {name[:42]:42s} {o['n']:3d} {o['ms'] / a.profile_steps:8.3f} "
                        f"{o['flops'] / t / 1e12:8.1f} {o['bytes'] / t / 1e9:8.1f} {100 * rt / t:6.1f}\n")

    if rank == 0:
        frames = a.batch * world * a.steps
        c5 = a.workload == "c5"
        out = {
            "metric": ("train frames/s (1024x2048 len-3 clips, two-stage extrapolation)" if c5
                       else "train frames/s (256x512 len-3 clips)"),
            "value": round(frames / dt, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt * 1e3 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.precision,
            "data": "synthetic (seeded Cityscapes-shaped triplets, HBM-resident); random-init HRNet, synthetic VGG19",
            "config": {"workload": (f"ExtraStage3Net (HRNet + SRNRefine + MSResAttnRefine, n_sc 3, stage3_prop) "
                                    f"int_9_len_3 train step {a.height}x{a.width} {a.precision}" if c5 else
                                    f"InterNet int_5_len_3 train step {a.height}x{a.width} {a.precision}"),
                       "per_gpu_batch": a.batch, "global_batch": a.batch * world, "parallelism": f"dp{world}",
                       "step": "hipGraph-captured" if a.graph else "eager, executor side-stream lanes"},
            "eager_ms_per_step": round(eager_dt * 1e3 / a.steps, 3),
            "roofline": roof,
            "loss_all": loss_all,
            "step_breakdown_ms": {k: round(v["ms"] / max(1, a.profile_steps), 3) for k, v in sorted(agg.items())},
        }
        at = [agg[c] for c in ("attn", "attn_bwd") if c in agg]
        if at:  # local-window attention of the stage-3 net (HBM-bound gathers / reductions)
            ms, by = sum(r["ms"] for r in at), sum(r["bytes"] for r in at)
            out["attn"] = {"ms_per_step": round(ms / a.profile_steps, 3), "launches_per_step": sum(r["n"] for r in at)
                           // a.profile_steps, "GBps": round(by / (ms * 1e-3) / 1e9, 1),
                           "frac": round(by / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
        if not c5:
            out["warp"] = warp_roofline(dev, a.batch, a.height, a.width)
            out["warp_1024x2048"] = warp_roofline(dev, a.batch, 1024, 2048, reps=5)  # BASELINE configs[4] frames
            out["clip_prep"] = clip_prep_roofline(dev, a.batch, a.height, a.width)
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_c5() if c5 else cpu_baseline(a.height, a.width)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
