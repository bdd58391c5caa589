"""Summarise a bench.py --ops-out table: ms per step by class and the ops that lose the most
time against their roofline (ms * (1 - roof%)).  usage: python tools/ops_lost.py ops.txt [N]"""
import sys

rows = []
for line in open(sys.argv[1]).read().splitlines()[1:]:
    p = line.split()
    cls, ms, roof, name = p[0], float(p[-4]), float(p[-1]), " ".join(p[1:-5])
    rows.append((cls, name, ms, roof, ms * (1 - roof / 100)))
print("total ms/step %.3f" % sum(r[2] for r in rows))
agg = {}
for r in rows:
    a = agg.setdefault(r[0], [0.0, 0.0])
    a[0] += r[2]
    a[1] += r[4]
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{k:12s} {v[0]:7.3f} ms  lost {v[1]:7.3f}")
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
for r in sorted(rows, key=lambda r: -r[4])[:n]:
    print(f"{r[0]:11s} {r[1][:40]:40s} {r[2]:6.3f} {r[3]:5.1f}% lost {r[4]:.3f}")
