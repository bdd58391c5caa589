"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) into per-kernel stats
(calls, total/avg duration, share), like the --stats CSV.  Usage:
    python tools/rocpd_summary.py <results.db> [out.csv]"""
import collections
import csv
import re
import sqlite3
import sys


def summarize(db):
    c = sqlite3.connect(db)
    rows = c.execute("select s.kernel_name, d.end - d.start, s.arch_vgpr_count, s.accum_vgpr_count, "
                     "s.group_segment_size from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
                     "on d.kernel_id = s.id").fetchall()
    agg = collections.OrderedDict()
    for name, ns, vg, ag, lds in rows:
        short = re.sub(r"\(.*", "", name)
        a = agg.setdefault(short, [0, 0, vg, ag, lds])
        a[0] += 1
        a[1] += ns
    tot = sum(v[1] for v in agg.values())
    out = sorted(((k, v[0], v[1], v[1] / v[0], 100.0 * v[1] / tot, v[2], v[3], v[4]) for k, v in agg.items()),
                 key=lambda r: -r[2])
    return out, tot


if __name__ == "__main__":
    out, tot = summarize(sys.argv[1])
    hdr = ["kernel", "calls", "total_ns", "avg_ns", "percent", "arch_vgpr", "accum_vgpr", "lds_bytes"]
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            w.writerows(out)
    for r in out[:40]:
        print(f"{r[4]:6.2f}% {r[1]:6d} calls {r[2]/1e6:9.3f} ms avg {r[3]/1e3:9.2f} us vgpr {r[5]}/{r[6]} lds {r[7]}  {r[0][:110]}")
    print("total ms", tot / 1e6)
