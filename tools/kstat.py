"""Mean duration (us) of the last N launches of each named kernel in rocprofv3 kernel traces.
usage: python tools/kstat.py DIR [DIR ...] -k name1 name2 ... [-n 100]"""
import argparse
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("-k", nargs="+", default=["render_bwd", "render_fwd<1", "gauss_sum", "gauss_live"])
ap.add_argument("-n", type=int, default=100)
a = ap.parse_args()
for d in a.dirs:
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if not f:
        print(d, "no trace")
        continue
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    out = []
    for k in a.k:
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if k in r["Kernel_Name"]]
        ds = ds[-a.n:]
        out.append(f"{k} {sum(ds) / max(len(ds), 1):.1f}")
    print(os.path.basename(d.rstrip('/')), " | ".join(out))
