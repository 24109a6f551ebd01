"""The precise tile cull's logf, round 5 against correctly rounded, on the CPU oracle.

The reference keeps a (tile, Gaussian) pair when max_contrib_power <= logf(co.w / (1/255)) with CUDA's logf
(rasterizer_impl.cu:151, 171).  Until round 5 the oracle and the kernels used a float polynomial (gs_logf_r5); now
both use the correctly rounded logf (gs_crlogf).  For the six workloads of tests/test_gpu_fullsize.py (same seeds,
same yaw views) this counts the keep decisions the two thresholds disagree on, and the opacities whose threshold
differs.  Plus the exhaustive check of gs_crlogf itself over every float in [2^-20, 256).

    python tools/logf_census.py --out profiles/r06_logf_census.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

WORKLOADS = [(100_000, 800, 800, 3), (1_000_000, 1920, 1080, 3), (5_000_000, 1920, 1080, 3),
             (1_000_000, 3840, 2160, 3), (5_000_000, 3840, 2160, 1), (2_000_000, 1280, 720, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="profiles/r06_logf_census.json")
    ap.add_argument("--quick", action="store_true", help="first two workloads only")
    args = ap.parse_args()
    from oracle import oracle as O
    from raster_util import yaw_view
    from dogs_amd.synthetic import make_scene
    O.set_threads(0)
    rec = {"what": "precise-cull keep decisions, round-5 gs_logf vs correctly rounded logf", "workloads": []}
    t0 = time.time()
    n_bad, bad = O.crlogf_check(0x35800000, 0x43800000)
    rec["crlogf_vs_logl_disagreements_2^-20_to_256"] = {"count": n_bad, "inputs": [float(x).hex() for x in bad],
                                                        "seconds": time.time() - t0}
    print(json.dumps(rec["crlogf_vs_logl_disagreements_2^-20_to_256"]), flush=True)
    tot = {}
    for n, W, H, views in (WORKLOADS[:2] if args.quick else WORKLOADS):
        base = make_scene(n, W, H, seed=1234)
        yaws = [0.0] + list(np.random.default_rng(1234).uniform(-10.0, 10.0, views - 1))
        for yaw in yaws:
            s = yaw_view(base, float(yaw))
            c = s.camera
            t = time.time()
            r = O.logf_census(s.means3D.numpy(), s.opacities.numpy(), c.world_to_camera.numpy(),
                              c.projective_matrix.numpy(), c.camera_center.numpy(), c.tanfovx, c.tanfovy, H, W,
                              s.scales.numpy(), s.rotations.numpy())
            r.update(n=n, W=W, H=H, yaw=float(yaw), seconds=round(time.time() - t, 2))
            rec["workloads"].append(r)
            for k in ("tested", "kept", "kept_only_r5", "kept_only_cr", "rendered", "threshold_differs"):
                tot[k] = tot.get(k, 0) + r[k]
            print(json.dumps(r), flush=True)
    rec["total"] = tot
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(tot))


if __name__ == "__main__":
    main()
