"""Local-step time of the ADMM block trainer (dogs_amd.admm_trainer.BlockTrainer) on one GPU, with the host time per
step, for kernel-trace profiling: python tools/trainer_bench.py [--n 1000000] [--steps 100]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--cprofile", action="store_true", help="print the host profile of the timed steps")
    ap.add_argument("--raster-only", action="store_true", help="time bench.py's raster view step instead")
    ap.add_argument("--alternate", action="store_true",
                    help="alternate the native step's routes (DG_TRAIN_UNFUSED on/off) every 10 steps")
    ap.add_argument("--bench-native", action="store_true",
                    help="time bench.py's native train step (no ADMM penalty, densification statistics on)")
    ap.add_argument("--bench-autograd", action="store_true",
                    help="time bench.py's autograd-route train step (the drop-in calls as the reference trainer makes)")
    ap.add_argument("--autograd-main-thread", action="store_true",
                    help="run the backward on the calling thread (torch.autograd.set_multithreading_enabled(False)) so "
                         "--cprofile sees the backward functions")
    args = ap.parse_args()
    if args.autograd_main_thread:
        torch.autograd.set_multithreading_enabled(False)
    from dogs_amd.admm import ADMMConfig
    from dogs_amd.admm_trainer import make_block
    dev = torch.device("cuda", 0)
    if args.bench_native or args.bench_autograd:
        import bench
        from dogs_amd.synthetic import make_scene
        s = make_scene(args.n, args.width, args.height, seed=1234).to(dev)
        cams = bench.make_cameras(args.width, args.height, bench.view_yaws(args.views), dev)
        ts = bench.TrainStep(s, cams, dev, 1234)
        step = ts.native() if args.bench_native else ts.step
    elif args.raster_only:
        import bench
        from dogs_amd.synthetic import make_scene
        s = make_scene(args.n, args.width, args.height, seed=1234).to(dev)
        cams = bench.make_cameras(args.width, args.height, bench.view_yaws(args.views), dev)
        g = torch.Generator().manual_seed(1234 + 99)
        gc = torch.randn((3, args.height, args.width), generator=g).to(dev)
        v = bench.Views(s, cams, gc, torch.zeros((1, args.height, args.width), device=dev), dev)
        step = v.step
    else:
        tr, _, _ = make_block(0, 1, args.n, args.width, args.height, args.views, 0.0, dev, admm=ADMMConfig())
        step = tr.local_step
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    host = []
    prof = None
    if args.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    blocks = {"unfused": [], "folded": []}
    t0 = time.perf_counter()
    tb = t0
    for i in range(args.steps):
        if args.alternate and i % 10 == 0:
            torch.cuda.synchronize()
            now = time.perf_counter()
            if i:
                blocks["unfused" if ((i // 10) - 1) % 2 == 0 else "folded"].append((now - tb) / 10)
            tb = now
            if (i // 10) % 2 == 0:
                os.environ["DG_TRAIN_UNFUSED"] = "1"
            else:
                os.environ.pop("DG_TRAIN_UNFUSED", None)
        h = time.perf_counter()
        step()
        host.append(time.perf_counter() - h)
    if args.alternate:
        torch.cuda.synchronize()
        blocks["unfused" if ((args.steps // 10) - 1) % 2 == 0 else "folded"].append((time.perf_counter() - tb) / 10)
        for k, v in blocks.items():
            if v:
                v = sorted(v)
                print(f"{k}: 10-step blocks {len(v)}, ms per step min {v[0] * 1e3:.4f} median {v[len(v) // 2] * 1e3:.4f}")
    torch.cuda.synchronize()
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof).sort_stats("tottime").print_stats(45)
    dt = (time.perf_counter() - t0) / args.steps
    host.sort()
    print(f"local step {dt * 1e3:.3f} ms ({1.0 / dt:.1f} views/s); host per step median {host[len(host) // 2] * 1e3:.3f}"
          f" ms, min {host[0] * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
