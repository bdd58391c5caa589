"""Step timeline from a rocprofv3 kernel trace (tools/gpu_trace.sh): steps are cut at the
weight-pack launch that opens every training step's forward; per step it prints the wall time,
the union of kernel-busy intervals (idle = wall - union), the busy time per queue (the executor's
weight lane runs on its own stream), and the largest idle gaps with the kernels around them.
usage: python tools/timeline.py <kernel_trace.csv> [--gaps N] [--classes]"""
import csv
import re
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"],
                         r.get("Stream_Id", "")))
    rows.sort()
    return rows


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    name = name.replace("dvie::", "")
    return name[:70]


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


CLASSES = [("wgrad", r"wgrad|head3_bwd|segenc_bwd"), ("wreduce", r"wreduce|colsum"),
           ("conv", r"conv|head3"), ("ew", r"ew_|ew1|ew_kernel"), ("loss", r"loss|ssim|l1|ce_|finalize|sum_f32"),
           ("pack", r"pack"), ("optim", r"adam")]


def klass(n):
    for c, rx in CLASSES:
        if re.search(rx, n):
            return c
    return "other"


def main():
    path = sys.argv[1]
    ngaps = int(sys.argv[sys.argv.index("--gaps") + 1]) if "--gaps" in sys.argv else 8
    rows = load(path)
    starts = [i for i, r in enumerate(rows) if re.search(r"pack_kernel", r[2])]
    if len(starts) < 3:
        print("fewer than 3 steps found", len(starts))
        return
    # the timed-region steps: the last full ones
    for k in range(len(starts) - 1):
        a, b = starts[k], starts[k + 1]
        seg = rows[a:b]
        t0, t1 = seg[0][0], rows[b][0]
        wall = (t1 - t0) / 1e6
        busy = union([(s, e) for s, e, *_ in seg]) / 1e6
        perq = defaultdict(float)
        percls = defaultdict(float)
        for s, e, n, q, st in seg:
            perq[q] += (e - s) / 1e6
            percls[klass(n)] += (e - s) / 1e6
        print(f"step {k}: wall {wall:.3f} ms, busy(union) {busy:.3f}, idle {wall - busy:.3f}, kernels {len(seg)}, "
              f"per-queue " + ", ".join(f"q{q} {v:.2f}" for q, v in sorted(perq.items())))
        if "--classes" in sys.argv:
            print("   " + ", ".join(f"{c} {v:.2f}" for c, v in sorted(percls.items(), key=lambda x: -x[1])))
    # gaps of the last step
    a, b = starts[-2], starts[-1]
    seg = rows[a:b + 1]
    gaps = []
    end = seg[0][1]
    for i in range(1, len(seg)):
        s = seg[i][0]
        if s > end:
            gaps.append(((s - end) / 1e3, i))
        end = max(end, seg[i][1])
    gaps.sort(reverse=True)
    print(f"largest idle gaps of the last step (us), total {sum(g for g, _ in gaps):.1f} us over {len(gaps)} gaps:")
    for g, i in gaps[:ngaps]:
        print(f"  {g:8.1f}  after {short(seg[i - 1][2])}  before {short(seg[i][2])}")


if __name__ == "__main__":
    main()
