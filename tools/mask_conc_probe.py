"""Masked pre-phase of the 2 x 2 test split: four processes training blocks 0-3 concurrently on the one GPU (as the
distributed test's ranks do) against the same blocks trained one after another in this process; prints, per block,
the first differing iteration.  --serial runs the children one at a time instead."""
import argparse
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--serial", action="store_true")
    a = ap.parse_args()
    from mask_det_probe import run_once
    with tempfile.TemporaryDirectory() as d:
        procs = []
        for b in range(4):
            cmd = [sys.executable, os.path.join(ROOT, "tools", "mask_det_probe.py"), "--child", os.path.join(d, f"{b}.pt"),
                   "--iters", str(a.iters), "--block", str(b)]
            p = subprocess.Popen(cmd)
            if a.serial:
                p.wait()
            procs.append(p)
        for p in procs:
            p.wait()
        kids = [torch.load(os.path.join(d, f"{b}.pt"), weights_only=False) for b in range(4)]
    for b in range(4):
        ref = run_once(a.iters, (b,))
        first = None
        for i, ((m1, e1, route), (m2, e2, _)) in enumerate(zip(ref, kids[b])):
            dm = [k for k, (x, y) in enumerate(zip(m1, m2)) if x.shape != y.shape or not torch.equal(x, y)]
            de = [k for k, (x, y) in enumerate(zip(e1, e2)) if not torch.equal(x, y)]
            if (dm or de) and first is None:
                first = (i + 1, route, dm, de)
        print(f"block {b}: first differing iteration {first}", flush=True)


if __name__ == "__main__":
    main()
