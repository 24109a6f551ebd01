"""Bit-level fingerprint of the bench workload's raster outputs, for comparing two library builds that should be
bit-identical (run once per build with DOGS_HIP_LIB, then compare the two JSON files).

usage: python tools/bitcmp.py OUT.json [--n N] [--views V]      compare: python tools/bitcmp.py --cmp A.json B.json
"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def digest(t) -> str:
    import torch
    return hashlib.sha256(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--cmp", nargs=2)
    args = ap.parse_args()
    if args.cmp:
        a, b = (json.load(open(p)) for p in args.cmp)
        bad = [k for k in a if a[k] != b.get(k)]
        print(f"{len(a)} tensors, {len(bad)} differ" + (": " + ", ".join(bad[:20]) if bad else ""))
        sys.exit(1 if bad or set(a) != set(b) else 0)
    import torch
    import bench
    import dogs_amd._lib as L
    L.load()
    dev = torch.device("cuda", 0)
    from dogs_amd.synthetic import make_scene
    W, H = 1920, 1080
    s = make_scene(args.n, W, H, seed=1234).to(dev)
    cams = bench.make_cameras(W, H, bench.view_yaws(args.views), dev)
    g = torch.Generator().manual_seed(1234 + 99)
    gc = torch.randn((3, H, W), generator=g).to(dev)
    gi = torch.randn((1, H, W), generator=g).to(dev) * 0.1
    v = bench.Views(s, cams, gc, gi, dev)
    res = {}
    for k in range(2 * args.views):  # twice round the batch: the adaptive capacity moves in the first pass
        out, grads = v.step()
        torch.cuda.synchronize()
        for i, t in enumerate(out):
            if torch.is_tensor(t) and t.numel() and i in (1, 2, 3, 4):
                res[f"v{k}.out{i}"] = digest(t)
        for i, t in enumerate(grads):
            if torch.is_tensor(t) and t.numel():
                res[f"v{k}.grad{i}"] = digest(t)
    json.dump(res, open(args.out, "w"), indent=0)
    print(f"{len(res)} tensors fingerprinted -> {args.out}")


if __name__ == "__main__":
    main()
