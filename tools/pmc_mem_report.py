"""Per-kernel vector-memory counters from tools/pmc_mem.sh: every counter summed over the
kernel's launches and divided by the launch count (per launch).  TA_BUSY_avr is averaged.
usage: python tools/pmc_mem_report.py <dir>"""
import collections
import csv
import glob
import re
import sys


def main(d):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.match(r"(?:void )?(?:dvie::)?([\w]+(?:<[^>]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:50]
            c = r["Counter_Name"]
            tot[k][c] += float(r["Counter_Value"])
            n[k][c].add((f, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
    for k in sorted(tot):
        print(k)
        for c in sorted(tot[k]):
            cnt = max(1, len(n[k][c]))
            print(f"    {c:40s} {tot[k][c] / cnt:16.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
