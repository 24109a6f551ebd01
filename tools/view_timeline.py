"""Per-kernel timeline of one timed view from a rocprofv3 kernel trace (tools/profile.sh output).
usage: python tools/view_timeline.py TRACE_CSV [view_index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_preprocess" in r["Kernel_Name"]]
v = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
st, en = idx[v], idx[v + 1]
t0 = int(rows[st]["Start_Timestamp"])
prev = None
tot = 0.0
for r in rows[st:en]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    tot += (e - s) / 1000
    print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f} gap {gap:5.1f}  {r['Kernel_Name'][:80]}")
    prev = e
print(f"kernel sum {tot:.1f} us, span {(prev - t0) / 1000:.1f} us")
