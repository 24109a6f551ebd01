"""Where the autograd-route train step (bench.TrainStep.step) spends its host time: cProfile over --steps steps (Python
functions, tottime), then torch.profiler with CPU activity only (aten ops and autograd nodes, self CPU time).
python tools/autograd_prof.py [--steps 60]"""
import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--n", type=int, default=1_000_000)
    args = ap.parse_args()
    import bench
    from dogs_amd.synthetic import make_scene
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    s = make_scene(args.n, W, H, seed=1234).to(dev)
    cams = bench.make_cameras(W, H, bench.view_yaws(8), dev)
    ts = bench.TrainStep(s, cams, dev, 1234)
    for _ in range(16):
        ts.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        ts.step()
    torch.cuda.synchronize()
    pr.disable()
    out = io.StringIO()
    st = pstats.Stats(pr, stream=out)
    st.sort_stats("tottime").print_stats(45)
    print(out.getvalue())
    out = io.StringIO()
    st = pstats.Stats(pr, stream=out)
    st.sort_stats("cumtime").print_stats(45)
    print(out.getvalue())
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(args.steps):
            ts.step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=60))


if __name__ == "__main__":
    main()
