"""Per-step kernel timelines of the native training step from tools/train_timeline.sh traces.
usage: python tools/train_timeline.py OUTDIR"""
import csv
import glob
import os
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def main(out):
    for route in ("unfused", "folded"):
        f = glob.glob(os.path.join(out, route, "**", "*kernel_trace.csv"), recursive=True)
        if not f:
            continue
        rows = load(f[0])
        idx = [i for i, r in enumerate(rows) if "k_activate_fwd" in r["Kernel_Name"]]
        spans = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000 for a, b in zip(idx, idx[1:])]
        spans = spans[len(spans) // 2:]
        print(f"== {route}: step span median {sorted(spans)[len(spans) // 2]:.1f} us over {len(spans)} steps")
        a, b = idx[-3], idx[-2]
        t0 = int(rows[a]["Start_Timestamp"])
        for r in rows[a:b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            q = r.get("Stream_Id") or r.get("Queue_Id", "?")
            print(f"  {(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f} q{q:>3}  {r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main(sys.argv[1])
