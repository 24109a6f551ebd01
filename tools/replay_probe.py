"""Is k_render_bwd tail-bound?  For each bench yaw view: the per-tile replay length (the tile's max contributor, which
the replay runs to), its distribution, and the longest-first schedule of those lengths over the chip's SIMDs against
the ideal (total / SIMDs).  Runs on the GPU box: python tools/replay_probe.py [--n 1000000] [--views 8]

Model (stated, not measured): a SIMD's VALU is shared by its resident waves, so a SIMD's load is the sum of its
tiles' lengths; the list-scheduling makespan is the largest SIMD load.  `lone` = longest tile / mean SIMD load: above
~1 the last wave alone on its SIMD sets the kernel's end."""
from __future__ import annotations

import argparse
import heapq
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def lpt(lengths, bins):
    """Greedy in the given order onto the least-loaded bin (the hardware dispatcher fills free slots in order)."""
    h = [0.0] * bins
    heapq.heapify(h)
    for x in lengths:
        heapq.heapreplace(h, h[0] + float(x))
    return max(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--simds", type=int, default=1024)
    args = ap.parse_args()
    import bench
    from dogs_amd import synthetic
    from raster_util import hip_image_state
    dev = torch.device("cuda:0")
    W, H = args.W, args.H
    s = synthetic.make_scene(args.n, W, H, seed=1234).to(dev)
    yaws = bench.view_yaws(args.views)
    cams = bench.make_cameras(W, H, yaws, dev)
    v = bench.Views(s, cams, None, None, dev)
    for k, c in enumerate(cams):
        for _ in range(3):  # settle the adaptive capacity
            out = v.forward(c)
        _, nc, mc, _ = hip_image_state(out, W, H, dev)
        L = mc.astype(np.float64)
        tot = L.sum()
        ideal = tot / args.simds
        order = np.sort(L)[::-1]
        span = lpt(order, args.simds)
        q = np.percentile(L, [50, 90, 99, 100]).round(0).tolist()
        print(f"view {k} yaw {yaws[k]:+.2f}: tiles {len(L)} replay sum {int(tot)} p50/p90/p99/max {q} "
              f"mean SIMD load {ideal:.0f} LPT span {span:.0f} ({span / ideal:.3f}x) lone {L.max() / ideal:.2f} "
              f"pixel n_contrib mean {nc.mean():.0f}")


if __name__ == "__main__":
    main()
