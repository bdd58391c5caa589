"""Per-kernel PMC report from tools/pmc_kernels.sh passes.

Per kernel template (summed over its launches in the 2+1-step bench run, then per launch):
duration (kernel-trace stats), MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8) (GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy counts cycles, 32 per
v_mfma_f32_32x32x16_bf16), HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB units; gfx950's
FETCH_SIZE reports half of wide streaming reads), GB/s over the traced duration, and the
wave-cycle split WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY (SQ_WAVE_CYCLES units), LDS bank
conflicts per LDS instruction.
usage: python tools/pmc_kernels_report.py <dir>"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.match(r"(?:void )?dvie::(\w+)<([^>]*)>", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name[:60]


def counters(d):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[k].add((f, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
    return tot, launches


def durations(d):
    out = {}
    for f in glob.glob(f"{d}/trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            out[k] = (int(r["Calls"]), float(r["AverageNs"]))
    return out


def main(d):
    tot, launches = counters(d)
    dur = durations(d)
    rows = []
    for k, c in tot.items():
        if k not in dur:
            continue
        calls, avg_ns = dur[k]
        n_pass = len(glob.glob(f"{d}/p[0-9]*/"))
        n_pmc = max(1, len({x for x in launches[k]}) // max(1, n_pass))  # each launch appears in every pass
        grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
        util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * grbm / 8.0) if grbm else 0.0
        hbm = (2.0 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0 / n_pmc
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        lds = c.get("SQ_INSTS_LDS", 0.0) or 1.0
        rows.append((calls * avg_ns, k, calls, avg_ns / 1e3, util, hbm / 1e6, hbm / avg_ns,
                     c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                     c.get("SQ_WAIT_INST_LDS", 0) / wc, c.get("SQ_LDS_BANK_CONFLICT", 0) / lds))
    rows.sort(reverse=True)
    print(f"{'kernel':48s} {'calls':>5s} {'avg_us':>8s} {'mfma%':>6s} {'MB/lnch':>8s} {'GB/s':>7s} "
          f"{'wait':>5s} {'wInst':>5s} {'activ':>5s} {'wLDS':>5s} {'bkcf/lds':>8s}")
    for _, k, calls, us, util, mb, gbs, wa, wi, ac, wl, bc in rows:
        print(f"{k[:48]:48s} {calls:5d} {us:8.1f} {100 * util:6.1f} {mb:8.1f} {gbs:7.0f} {wa:5.2f} {wi:5.2f} "
              f"{ac:5.2f} {wl:5.2f} {bc:8.3f}")
    print()
    print(f"{'kernel (instructions per wave)':48s} {'waves':>9s} {'VALU':>8s} {'VMEM_RD':>8s} {'VMEM_WR':>8s} {'LDS':>8s} "
          f"{'SALU':>8s}")
    for _, k, *_ in rows:
        c = tot[k]
        wv = c.get("SQ_WAVES", 0.0) or 1.0
        print(f"{k[:48]:48s} {wv:9.0f} {c.get('SQ_INSTS_VALU', 0) / wv:8.1f} {c.get('SQ_INSTS_VMEM_RD', 0) / wv:8.1f} "
              f"{c.get('SQ_INSTS_VMEM_WR', 0) / wv:8.1f} {c.get('SQ_INSTS_LDS', 0) / wv:8.1f} "
              f"{c.get('SQ_INSTS_SALU', 0) / wv:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
