"""GPU idle gaps inside a training step, from a rocprofv3 kernel trace (steps delimited by k_preprocess): per step the
span, the kernels' busy time (union of intervals) and the idle gaps between consecutive kernels, reported as medians
per (previous kernel -> next kernel) pair.  Busy well below the span means the host (or a sync) starves the GPU.
usage: python tools/step_gaps.py TRACE_DIR [--top 15]"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("gs::", "")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--skip", type=int, default=4, help="leading steps to drop (warm-up)")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.out, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_preprocess" in r["Kernel_Name"]]
    spans, busy, gaps = [], [], collections.defaultdict(list)
    nsteps = 0
    for a0, b0 in list(zip(idx, idx[1:]))[a.skip:]:
        seg = rows[a0:b0 + 1]
        t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["Start_Timestamp"])
        spans.append((t1 - t0) / 1e3)
        bz, end = 0, t0
        step_gaps = collections.defaultdict(float)
        for r, nx in zip(seg[:-1], seg[1:]):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            bz += max(0, e - max(s, end))
            end = max(end, e)
            g = int(nx["Start_Timestamp"]) - end
            if g > 0:
                step_gaps[(short(r["Kernel_Name"]), short(nx["Kernel_Name"]))] += g / 1e3
        busy.append(bz / 1e3)
        for k, v in step_gaps.items():
            gaps[k].append(v)
        nsteps += 1
    print(f"{nsteps} steps: span median {statistics.median(spans):.1f} us, kernel busy median "
          f"{statistics.median(busy):.1f} us, idle {statistics.median(spans) - statistics.median(busy):.1f} us")
    tot = sorted(((sum(v) / nsteps, k, len(v)) for k, v in gaps.items()), reverse=True)
    for m, (p, n), c in tot[:a.top]:
        print(f"  {m:8.1f} us/step  {p} -> {n}  (in {c} steps)")
    kern = collections.defaultdict(float)
    for r in rows[idx[a.skip]:idx[-1]]:
        kern[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("kernel time per step:")
    for k, v in sorted(kern.items(), key=lambda kv: -kv[1])[:30]:
        print(f"  {v / nsteps:8.1f} us  {k}")


if __name__ == "__main__":
    main()
