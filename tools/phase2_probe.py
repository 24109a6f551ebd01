"""Where does phase 2 come from?  For each bench yaw view: the tiles phase 1 left unfinished (they carry phase-2
instances), their phase-1 prefix length n1, their full list length n (depth-prefix binning off) and the tile's max
contributor over the full list; aggregated per supertile of S x S tiles, and the tile-rect area per supertile.
Runs on the GPU box: python tools/phase2_probe.py [--n 1000000] [--S 8]"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--S", type=int, default=8)
    ap.add_argument("--views", type=int, default=8)
    args = ap.parse_args()
    import bench
    from dogs_amd import synthetic
    from dogs_amd.diff_gaussian_rasterization import _C
    from raster_util import hip_image_state, hip_sorted_instances
    dev = torch.device("cuda:0")
    W, H, S = args.W, args.H, args.S
    tx, ty = (W + 15) // 16, (H + 15) // 16
    T = tx * ty
    s = synthetic.make_scene(args.n, W, H, seed=1234).to(dev)
    yaws = bench.view_yaws(args.views)
    cams = bench.make_cameras(W, H, yaws, dev)
    v = bench.Views(s, cams, None, None, dev)
    tile_st = (np.arange(T) // tx // S) * ((tx + S - 1) // S) + (np.arange(T) % tx) // S
    for k, c in enumerate(cams):
        for _ in range(3):  # settle the adaptive capacity
            out = v.forward(c)
        t_h, _, e1 = hip_sorted_instances(out, W, H, dev, args.n)
        n1 = np.bincount(t_h[:e1], minlength=T)
        n2 = np.bincount(t_h[e1:], minlength=T)
        old = _C.set_prefix_per_tile(-1)
        try:
            ref = v.forward(c)
            t_f, _, ef = hip_sorted_instances(ref, W, H, dev, args.n)
            _, _, mc, _ = hip_image_state(ref, W, H, dev)
        finally:
            _C.set_prefix_per_tile(old)
        nf = np.bincount(t_f[:ef], minlength=T)
        unf = n2 > 0
        st_full = np.bincount(tile_st, weights=nf)
        st_unf = np.bincount(tile_st, weights=unf.astype(float))
        st_tiles = np.bincount(tile_st)
        print(f"view {k} yaw {yaws[k]:+.2f}: E1 {e1} E2 {len(t_h) - e1} K {ef} tiles with phase-2 instances {unf.sum()}")
        if unf.any():
            q = lambda a: np.percentile(a, [0, 50, 90, 99, 100]).round(0).tolist()  # noqa: E731
            print(f"  unfinished: n1 {q(n1[unf])}  n_full {q(nf[unf])}  max_contrib {q(mc[unf])}  n1==0: "
                  f"{int((n1[unf] == 0).sum())}  sum n_full {int(nf[unf].sum())}")
            fin = ~unf & (nf > 0)
            print(f"  finished:   n1 {q(n1[fin])}  n_full {q(nf[fin])}  max_contrib {q(mc[fin])}")
            sts = np.nonzero(st_unf)[0]
            dens = st_full[sts] / st_tiles[sts]
            print(f"  supertiles with unfinished tiles: {len(sts)} of {len(st_tiles)}; their full instances per tile "
                  f"{q(dens)}; all supertiles {q(st_full / st_tiles)}")
            # how many instances a 'complete the supertile' rule would add, by density level
            for L in (64, 128, 256, 448, 672, 1008):
                pick = (st_full / st_tiles) <= L
                covered = unf & pick[tile_st]
                extra = (nf - n1)[pick[tile_st]].sum()
                print(f"    complete supertiles with <= {L:4d} inst/tile: covers {int(covered.sum())}/{int(unf.sum())} "
                      f"unfinished tiles, adds {int(extra)} instances ({extra / max(e1, 1):.2%} of E1)")


if __name__ == "__main__":
    main()
