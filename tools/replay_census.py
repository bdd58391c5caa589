"""Kernel census of hipGraph replays of the bench step (BASELINE configs[1]).

    python tools/replay_census.py run [replays]        (under rocprofv3 --kernel-trace)
    python tools/replay_census.py report <kernel_trace.csv>
    python tools/replay_census.py aten [H W batch]     (no profiler: aten ops of one eager step)

`run` builds the bench trainer (InterNet 256x512 bf16, batch 8), captures the step
(runners/graph.py) and replays it, each replay preceded by a marker kernel
(torch.cuda._sleep).  `report` splits the trace at the markers and prints, per replay, the
kernel count by family -- in particular every PyTorch-native (at::native) kernel left
inside the captured step."""
import collections
import csv
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(replays):
    import torch
    sys.argv = [sys.argv[0]]
    import bench
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer
    from deep_video_interpolation_extrapolation_amd.runners.graph import GraphedStep
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    args = default_args("INTER", syn_type="inter", interval=5, mode="xs2xs", vid_length=1, train_coarse=True,
                        batch_size=8, input_h=256, input_w=512, precision="bf16", synthetic=8, num_workers=0,
                        split="train")
    torch.manual_seed(args.seed)
    tr = InterTrainer(args)
    data = bench.make_batch(8, 256, 512, dev, 0)
    gs = GraphedStep(tr, data, warmup=2)
    torch.cuda.synchronize()
    for _ in range(replays):
        torch.cuda._sleep(2000)  # marker
        gs.step()
    torch.cuda._sleep(2000)
    torch.cuda.synchronize()
    print("replays", replays)


def aten(H=256, W=512, B=8):
    """Every aten op one eager bench step dispatches (views and metadata ops excluded), with
    the Python frame in this package that issued it: the PyTorch glue left around the
    native plan launches."""
    import traceback
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode
    sys.argv = [sys.argv[0]]
    import bench
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    args = default_args("INTER", syn_type="inter", interval=5, mode="xs2xs", vid_length=1, train_coarse=True,
                        batch_size=B, input_h=H, input_w=W, precision="bf16", synthetic=B, num_workers=0,
                        split="train")
    torch.manual_seed(args.seed)
    tr = InterTrainer(args)
    data = bench.make_batch(B, H, W, dev, 0)
    tr.step(data)
    tr.step(data)
    torch.cuda.synchronize()
    skip = ("view", "_unsafe_view", "as_strided", "alias", "detach", "t.default", "expand", "slice", "select",
            "unsqueeze", "squeeze", "permute", "transpose", "split", "unbind", "_to_copy", "lift_fresh",
            "is_same_size", "empty", "_local_scalar_dense", "item")
    seen = collections.Counter()
    where = {}

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func)
            if not any(name.startswith("aten." + k) for k in skip):
                fr = [f for f in traceback.extract_stack()
                      if "deep_video_interpolation_extrapolation_amd" in f.filename]
                loc = f"{os.path.basename(fr[-1].filename)}:{fr[-1].lineno}" if fr else "?"
                shp = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)][:2]
                seen[(name, loc)] += 1
                where.setdefault((name, loc), shp)
            return func(*args, **(kwargs or {}))

    with Log():
        tr.step(data)
    torch.cuda.synchronize()
    print(f"aten ops of one eager step at {B}x{H}x{W}: {sum(seen.values())}")
    for (name, loc), n in seen.most_common():
        print(f"    {n:4d}  {name:40s} {loc:28s} {where[(name, loc)]}")


def family(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"<.*", "", n).replace("void ", "")
    return n


def report(path):
    rows = list(csv.DictReader(open(path)))
    key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "sleep" in r[key].lower() or "spin" in r[key].lower()]
    print(f"{len(rows)} kernels, {len(marks)} markers")
    for a, b in zip(marks, marks[1:]):
        seg = rows[a + 1:b]
        fam = collections.Counter(family(r[key]) for r in seg)
        t = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e6
        span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6 if seg else 0
        nat = [r for r in seg if "at::" in r[key]]
        nt = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in nat) / 1e3
        print(f"replay: {len(seg)} kernels, busy {t:.3f} ms, span {span:.3f} ms; PyTorch-native kernels: "
              f"{len(nat)} ({nt:.1f} us)")
        for k, v in fam.most_common():
            print(f"    {v:5d}  {k}")
        for k, v in collections.Counter(re.sub(r", std::array.*|\(int,.*", "", r[key])[:160] for r in nat).most_common():
            print(f"    native {v:3d}  {k}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
    elif sys.argv[1] == "aten":
        aten(*[int(v) for v in sys.argv[2:5]])
    else:
        report(sys.argv[2])
