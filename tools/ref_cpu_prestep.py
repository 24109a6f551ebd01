"""the reference's own PyTorch-CPU pre-steps for the preprocess stage -- eval_sh (colour from SH)
and the covariance L L^T (rotation_mat_left_multiply_scale_mat) -- imported by file path from /root/reference (this
container only; the GPU box has no reference), timed on the bench's synthetic 1e6-Gaussian scene, all threads and one.
usage: python tools/ref_cpu_prestep.py [n]  -> prints one JSON line"""
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = "/root/reference/conerf"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    from dogs_amd.synthetic import make_scene
    sh_utils = _load("ref_sh_utils", f"{REF}/model/gaussian_fields/sh_utils.py")
    gutils = _load("ref_gs_utils", f"{REF}/model/gaussian_fields/utils.py")
    s = make_scene(n)
    feats = torch.cat([s.dc, s.sh], dim=1).transpose(1, 2)            # [N, 3, 16]
    campos = s.camera.camera_center
    dirs = s.means3D - campos
    dirs = dirs / dirs.norm(dim=1, keepdim=True)

    def step():
        rgb = torch.clamp_min(sh_utils.eval_sh(3, feats, dirs) + 0.5, 0.0)
        L = gutils.rotation_mat_left_multiply_scale_mat(s.scales, s.rotations)
        cov = L @ L.transpose(1, 2)
        return rgb, cov

    out = {"n": n, "what": "reference eval_sh(3) + clamp and L L^T covariance on torch CPU (gaussian_fields/sh_utils.py:57, "
                           "utils.py:70)", "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0]
           .strip(" :\t")}
    for threads in (os.cpu_count(), 1):
        torch.set_num_threads(threads)
        step()
        t = time.perf_counter()
        reps = 3
        for _ in range(reps):
            step()
        out[f"seconds_{threads}_threads"] = round((time.perf_counter() - t) / reps, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
