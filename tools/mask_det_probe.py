"""Where the masked pre-phase stops being repeatable: block 0 of the 2 x 2 test split trained with the appearance mask
(GaussianSplatTrainer, the ADMM test config) twice in this process and once in a child process; prints which tensors
differ.  python tools/mask_det_probe.py [--child OUT]"""
import argparse
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run_once(iters, blocks=(0,)):
    from test_gpu_admm_run import _cfg, _scenes
    from dogs_amd.admm_run import pre_phase_trainer
    dev = torch.device("cuda", 0)
    with tempfile.TemporaryDirectory() as tmp:
        scenes = _scenes(dev, tmp)
    for b in blocks[:-1]:       # warm the process on the earlier blocks, as run_sequential does
        pre = pre_phase_trainer(_cfg(True), scenes[b], dev, 3)
        for _ in range(iters):
            pre.train_iteration()
        pre.sync()
    pre = pre_phase_trainer(_cfg(True), scenes[blocks[-1]], dev, 3)
    out = []
    for i in range(iters):
        pre.train_iteration()
        pre.sync()
        out.append(([t.detach().cpu().clone() for t in pre.model.get_all_properties()],
                    [p.detach().cpu().clone() for p in pre.mask.parameters()], pre.logs[-1].route))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", default=None)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--block", type=int, default=1)
    a = ap.parse_args()
    if a.child:
        torch.save(run_once(a.iters, (a.block,)), a.child)
        return
    r1 = run_once(a.iters, tuple(range(a.block + 1)))      # warm: blocks 0 .. block-1 trained first
    r2 = run_once(a.iters, (a.block,))
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "c.pt")
        subprocess.run([sys.executable, __file__, "--child", f, "--iters", str(a.iters), "--block", str(a.block)],
                       check=True)
        r3 = torch.load(f, weights_only=False)
    for name, other in (("same process (block alone after the warm run)", r2), ("cold child process", r3)):
        first = None
        for i, ((m1, e1, route), (m2, e2, _)) in enumerate(zip(r1, other)):
            dm = [k for k, (x, y) in enumerate(zip(m1, m2)) if x.shape != y.shape or not torch.equal(x, y)]
            de = [k for k, (x, y) in enumerate(zip(e1, e2)) if not torch.equal(x, y)]
            if (dm or de) and first is None:
                first = (i + 1, route, dm, de)
        print(f"{name}: first differing iteration {first} (iteration, route, model tensors, embedding params)", flush=True)
    print("routes:", [r[2] for r in r1])


if __name__ == "__main__":
    main()
