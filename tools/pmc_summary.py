"""Summarise rocprofv3 output (rocpd .db or --output-format csv) of tools/profile.sh into per-kernel figures.

usage: python tools/pmc_summary.py OUTDIR      (OUTDIR/trace = kernel trace, OUTDIR/pmc* = counter passes)

Per kernel (averaged per dispatch): duration, waves, instructions per wave, VALU utilisation
(SQ_ACTIVE_INST_VALU is in quad-cycles, summed over waves: x4 / (duration cycles x 1024 SIMDs)), the wait
fraction and HBM bytes (FETCH_SIZE x 2 on gfx950 per MI355X_MICROARCH.md's rocprofv3 section, + WRITE_SIZE;
both in KB).
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict

CLOCK_GHZ = 2.4
SIMDS = 1024


def _short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "gs::", "__amd_rocclr_"):
        n = n.replace(p, "")
    return n[:48]


def load_counters(root):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [value per dispatch]
    for f in glob.glob(os.path.join(root, "pmc*", "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        per = defaultdict(float)
        names = {}
        for d, k, cn, v in con.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            per[(d, cn)] += v
            names[d] = k
        for (d, cn), v in per.items():
            acc[_short(names[d])][cn].append(v)
    for f in glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, cn), v in per.items():
            acc[_short(names[d])][cn].append(v)
    return acc


def load_durations(root):
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "trace", "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        for name, d in con.execute("select name, duration from kernels"):
            dur[_short(name)].append(d / 1000.0)
    for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[_short(r["Name"])].append(float(r["AverageNs"]) / 1000.0)
    return dur


def avg(v):
    return sum(v) / len(v) if v else 0.0


def main(root):
    acc = load_counters(root)
    dur = load_durations(root)
    rows = []
    for k in set(acc) | set(dur):
        c = {n: avg(v) for n, v in acc.get(k, {}).items()}
        d = avg(dur.get(k, []))
        waves = c.get("SQ_WAVES", 0.0)
        cyc = d * 1e-6 * CLOCK_GHZ * 1e9
        r = {"kernel": k, "us": d, "calls": len(dur.get(k, [])), "waves": waves}
        if waves:
            for n, s in (("SQ_INSTS_VALU", "valu/w"), ("SQ_INSTS_SALU", "salu/w"), ("SQ_INSTS_LDS", "lds/w"),
                         ("SQ_INSTS_VMEM_RD", "vmrd/w"), ("SQ_INSTS_VMEM_WR", "vmwr/w")):
                r[s] = c.get(n, 0.0) / waves
        if cyc and "SQ_ACTIVE_INST_VALU" in c:
            r["valu_util"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * SIMDS)
        if c.get("SQ_WAVE_CYCLES"):
            r["wait"] = c.get("SQ_WAIT_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            mb = (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) / 1024.0
            r["hbm_MB"] = mb
            if d:
                r["GB/s"] = mb * 1e-3 / (d * 1e-6)
        rows.append(r)
    rows.sort(key=lambda r: -r["us"] * max(r["calls"], 1))
    cols = ["kernel", "us", "calls", "waves", "valu/w", "salu/w", "lds/w", "vmrd/w", "valu_util", "wait", "hbm_MB", "GB/s"]
    print("  ".join(f"{c:>9s}" if c != "kernel" else f"{c:48s}" for c in cols))
    for r in rows:
        out = []
        for c in cols:
            v = r.get(c)
            if c == "kernel":
                out.append(f"{v:48s}")
            elif v is None:
                out.append(f"{'-':>9s}")
            elif isinstance(v, float) and abs(v) < 10:
                out.append(f"{v:9.3f}")
            else:
                out.append(f"{v:9.0f}")
        print("  ".join(out))


if __name__ == "__main__":
    main(sys.argv[1])
