"""Per-step kernel timelines of the native training step from tools/train_timeline.sh traces (steps delimited by
k_preprocess, the first launch of a step since the activations moved into it).
usage: python tools/train_timeline.py OUTDIR"""
import csv
import glob
import os
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def by_kind(out):
    """One trace holding both routes (trainer_bench.py --alternate): steps classified by their kernels."""
    f = glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True)
    rows = load(f[0])
    idx = [i for i, r in enumerate(rows) if "k_preprocess" in r["Kernel_Name"]]
    spans = {"unfused": [], "folded": []}
    ksum = {"unfused": [], "folded": []}
    for a, b in zip(idx, idx[1:]):
        names = " ".join(r["Kernel_Name"] for r in rows[a:b])
        kind = "unfused" if "k_activate_bwd" in names else "folded"
        spans[kind].append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000)
        ksum[kind].append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b]) / 1000)
    for k in spans:
        sp, ks = sorted(spans[k]), sorted(ksum[k])
        if sp:
            print(f"{k}: {len(sp)} steps, span median {sp[len(sp) // 2]:.1f} us, kernel sum median {ks[len(ks) // 2]:.1f} us")


def main(out):
    if os.environ.get("BY_KIND"):
        by_kind(out)
        return
    for route in ("unfused", "folded"):
        f = glob.glob(os.path.join(out, route, "**", "*kernel_trace.csv"), recursive=True)
        if not f:
            continue
        rows = load(f[0])
        idx = [i for i, r in enumerate(rows) if "k_preprocess" in r["Kernel_Name"]]
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
