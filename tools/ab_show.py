"""Print value and per-phase times of every bench log in a directory (same-box A/B experiments)."""
import glob
import json
import sys

for f in sorted(glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab") + "/*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        print(f, "no JSON line")
        continue
    ph = " ".join(f"{k}={v * 1000:.0f}" for k, v in d.get("phases_ms", {}).items())
    print(f"{f.split('/')[-1]:14s} {d['value']:8.1f}  {ph}")
