"""Bitwise repeatability of the appearance embedding's forward and backward across processes: N child processes
(run concurrently, as the ADMM ranks sharing a GPU) and this process compute the same masked forward / backward on
the same seeded inputs; prints which outputs differ from this process's.
python tools/embed_det_probe.py [--W 160 --H 120 --children 4]"""
import argparse
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def once(W, H):
    from dogs_amd.masks import AppearanceEmbedding, downsample_image
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    net = AppearanceEmbedding(4).to(dev)
    with torch.no_grad():
        net.appearance_embedding.normal_(0.0, 0.3)
    g = torch.Generator().manual_seed(6)
    gt = torch.rand((3, H, W), generator=g).to(dev)
    dm = torch.randn((3, H, W), generator=g).to(dev)
    small = downsample_image(gt, 32).contiguous()
    out = {}
    m = net(small, 1, (H, W))
    m.backward(dm)
    out["mask"] = m.detach().cpu()
    for k, p in net.named_parameters():
        out["grad." + k] = p.grad.detach().cpu()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--W", type=int, default=160)
    ap.add_argument("--H", type=int, default=120)
    ap.add_argument("--children", type=int, default=4)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        torch.save(once(a.W, a.H), a.child)
        return
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, __file__, "--child", os.path.join(d, f"{i}.pt"), "--W", str(a.W),
                                   "--H", str(a.H)]) for i in range(a.children)]
        mine = once(a.W, a.H)
        for p in procs:
            assert p.wait() == 0
        for i in range(a.children):
            other = torch.load(os.path.join(d, f"{i}.pt"), weights_only=True)
            bad = [k for k in mine if not torch.equal(mine[k], other[k])]
            print(f"child {i}: {len(bad)} of {len(mine)} differ {bad}", flush=True)


if __name__ == "__main__":
    main()
