"""HBM bytes per launch of the bench's conv kernel families from the PMC passes of
tools/pmc_bench.sh.  gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE
(kilobytes) reports half the bytes of wide coalesced streaming reads -> x2; WRITE_SIZE
(kilobytes) is exact for 16-B streaming stores.  Writes <dir>/traffic.json:
{family: {"launches": n, "read_bytes": r, "write_bytes": w, "bytes_per_launch": b}}.
usage: python tools/pmc_traffic.py <dir>"""
import collections
import csv
import glob
import json
import re
import sys

FAM = [("conv", r"head3_bwd_kernel|segenc_fwd_kernel|conv_narrow_kernel|conv_h8_kernel|conv_halo_kernel|conv_ws_kernel|conv_strip_kernel|conv_nk_kernel|conv1x1_kernel|conv1x1_persist_kernel|conv1x1_ring_kernel|conv_s2_kernel|conv_igemm_kernel"),
       ("wgrad", r"segenc_bwd_kernel|wgrad_halo_kernel|wgrad_kernel|wgrad_wide_kernel")]


def family(name):
    for f, rx in FAM:
        if re.search(rx, name):
            return f
    return None


def load(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{d}/{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            fam = family(r["Kernel_Name"])
            if fam:
                vals[fam].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main(d):
    rd, wr = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    out = {}
    for fam in sorted(set(rd) | set(wr)):
        n = max(len(rd.get(fam, [])), len(wr.get(fam, [])))
        r = 2.0 * sum(rd.get(fam, [])) / max(1, len(rd.get(fam, [])))
        w = sum(wr.get(fam, [])) / max(1, len(wr.get(fam, [])))
        out[fam] = {"launches": n, "read_bytes": r, "write_bytes": w, "bytes_per_launch": r + w}
        print(f"{fam:6s} launches {n:5d}  read {r / 1e6:9.2f} MB  write {w / 1e6:9.2f} MB  per launch "
              f"{(r + w) / 1e6:9.2f} MB  (FETCH_SIZE x2 gfx950 correction)")
    json.dump(out, open(f"{d}/traffic.json", "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
