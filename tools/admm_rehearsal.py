"""The bench's ADMM leg alone (bench.admm_leg: pre-phase with densification, phase entry, ADMM rounds, then rank 0's
sequential baseline and the bit-for-bit comparison of rank 0's block), for rehearsals at scales the raster leg of
bench.py would not fit beside (several gloo ranks sharing one GPU).  Launch under torch.distributed.run, e.g.
  DOGS_BENCH_SHARE_DEVICE=1 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port 29533 tools/admm_rehearsal.py --points 13000000 --width 3840 --height 2160
Rank 0 prints one JSON line."""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1_000_000, help="points per block")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--admm-pre", type=int, default=100)
    ap.add_argument("--admm-rounds", type=int, default=1)
    ap.add_argument("--admm-interval", type=int, default=100)
    args = ap.parse_args()
    import bench
    rank = int(os.environ.get("RANK", "0"))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DOGS_BENCH_SHARE_DEVICE") == "1":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if ws > 1:
        dist.init_process_group(os.environ.get("DOGS_DIST_BACKEND", "gloo"))
    dev = torch.device("cuda", local)
    out = bench.admm_leg(args, ws, rank, dev, args.points, args.width, args.height)
    if rank == 0:
        print(json.dumps({"world": ws, "points_per_block_arg": args.points, "width": args.width,
                          "height": args.height, "admm": out}), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
