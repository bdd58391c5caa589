"""Kernels per EAGER bench step, by name, from two rocprofv3 --kernel-trace --stats runs of
the same bench command that differ only in --steps (tools/gpu_census.sh): per-step count =
(calls in the long run - calls in the short run) / (step difference), so setup, warm-up and
profiling launches cancel.  Lists every kernel that is not one of libdvie's (dvie::) -- the
PyTorch-native kernels the timed step still launches.
usage: python tools/eager_census.py <short kernel_stats.csv> <long kernel_stats.csv> <step difference>"""
import csv
import sys


def counts(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[r["Name"]] = out.get(r["Name"], 0) + int(r["Calls"])
    return out


def main(a, b, dsteps):
    ca, cb = counts(a), counts(b)
    per = {k: (cb.get(k, 0) - ca.get(k, 0)) / dsteps for k in set(ca) | set(cb)}
    per = {k: v for k, v in per.items() if abs(v) > 1e-9}
    dv = {k: v for k, v in per.items() if "dvie::" in k}
    other = {k: v for k, v in per.items() if "dvie::" not in k}
    print(f"kernels per eager step: {sum(per.values()):.1f} total, {sum(dv.values()):.1f} libdvie, "
          f"{sum(other.values()):.1f} other (PyTorch / runtime)")
    for k, v in sorted(other.items(), key=lambda kv: -kv[1]):
        print(f"  {v:6.2f}  {k[:160]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]))
