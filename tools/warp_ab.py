"""Same-process A/B of a warp-forward launch knob (read per launch by dvie_warp_fwd):
alternates the values over several rounds at 256x512 and 1024x2048 (batch 8) and prints
the median forward time and HBM fraction of each.

usage: python tools/warp_ab.py VAR A B [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    var, vals = sys.argv[1], sys.argv[2:4]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    dev = torch.device("cuda:0")
    res = {(v, s): [] for v in vals for s in ((256, 512), (1024, 2048))}
    for _ in range(rounds):
        for v in vals:
            os.environ[var] = v
            for s in ((256, 512), (1024, 2048)):
                r = bench.warp_roofline(dev, 8, s[0], s[1], reps=20 if s[0] == 256 else 10)
                res[(v, s)].append((r["fwd_ms"], r["fwd_frac"], r["bwd_ms"]))
    for (v, s), xs in res.items():
        f = statistics.median(x[0] for x in xs)
        fr = statistics.median(x[1] for x in xs)
        b = statistics.median(x[2] for x in xs)
        print(f"{var}={v} {s[0]}x{s[1]} fwd {f * 1e3:.1f} us frac {fr:.4f}  bwd {b * 1e3:.1f} us")


if __name__ == "__main__":
    main()
