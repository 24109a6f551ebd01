"""torch.profiler view of bench.py's autograd-route train step (the drop-in calls): which torch / library op issues
each kernel, and its host (CPU) time: python tools/autograd_prof.py [--steps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1_000_000)
    a = ap.parse_args()
    import bench
    from dogs_amd.synthetic import make_scene
    dev = torch.device("cuda", 0)
    s = make_scene(a.n, 1920, 1080, seed=1234).to(dev)
    cams = bench.make_cameras(1920, 1080, bench.view_yaws(8), dev)
    ts = bench.TrainStep(s, cams, dev, 1234)
    for _ in range(10):
        ts.step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(a.steps):
            ts.step()
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print(ka.table(sort_by="self_cpu_time_total", row_limit=45, max_name_column_width=70))
    print(ka.table(sort_by="self_device_time_total", row_limit=45, max_name_column_width=70))


if __name__ == "__main__":
    main()
