"""Group a rocprofv3 --stats kernel_stats.csv into the kernel families bench.py reports
(conv = forward + data-gradient launches of every conv kernel; wgrad; pointwise; loss ...)
so the rocprof average launch duration can be checked against bench.py's HIP-event figure.
usage: python tools/prof_family.py <kernel_stats.csv> [steps]"""
import csv
import re
import sys

FAMILIES = [("conv (fwd+dgrad)", r"conv_halo_kernel|conv_ws_kernel|conv1x1_kernel|conv_igemm_kernel"),
            ("wgrad", r"wgrad_halo_kernel|wgrad_kernel"),
            ("wreduce", r"wreduce_kernel"),
            ("colsum", r"colsum_kernel"),
            ("pointwise", r"ew_kernel"),
            ("loss", r"l1gdl|ssim|ce_|loss|finalize|l1nhwc"),
            ("pack", r"pack_kernel"),
            ("adamax", r"adamax")]


def main(path, steps=None):
    fam = {}
    total = 0
    for row in csv.DictReader(open(path)):
        name, calls, ns = row["Name"], int(row["Calls"]), float(row["TotalDurationNs"])
        total += ns
        key = "other"
        for f, rx in FAMILIES:
            if re.search(rx, name):
                key = f
                break
        a = fam.setdefault(key, [0, 0.0])
        a[0] += calls
        a[1] += ns
    print(f"{'family':18s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'share':>6s}" +
          (f" {'calls/step':>10s} {'ms/step':>8s}" if steps else ""))
    for k, (c, ns) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        line = f"{k:18s} {c:7d} {ns / 1e6:10.3f} {ns / c / 1e3:9.2f} {100 * ns / total:5.1f}%"
        if steps:
            line += f" {c / steps:10.1f} {ns / 1e6 / steps:8.3f}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
