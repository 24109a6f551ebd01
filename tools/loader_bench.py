"""Image path timing: 1080p RGB images from a decoded .npy cache to float CHW on the GPU.
  native: dogs_amd.loader.ImageReader (C++ readers -> pinned slots -> u8 async copy -> GPU conversion)
  reference-style: the reference's ImageReader flow without the decode -- Python worker threads load the u8 array
  and make the float32 HWC CPU tensor (read_image), the consumer copies it to the device and permutes to CHW.
usage: python tools/loader_bench.py [n_images] [threads]"""
import os
import queue
import sys
import tempfile
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dogs_amd.loader import ImageReader  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dev = torch.device("cuda:0")
d = tempfile.mkdtemp()
rng = np.random.default_rng(0)
paths = []
for i in range(8):  # 8 distinct files, cycled (page-cache resident, as a warm epoch)
    p = os.path.join(d, f"im{i}.png")
    np.save(p + ".npy", rng.integers(0, 256, (1080, 1920, 3), dtype=np.uint8))
    paths.append(p)
image_list = [paths[i % 8] for i in range(n)]

r = ImageReader(max_size=16, max_num_threads=threads, image_list=image_list, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
r.add_task(None)
for _ in range(n):
    _, img = r.get_image()
    chw = img.permute(2, 0, 1)
torch.cuda.synchronize()
native = n / (time.perf_counter() - t0)
r.safe_exit()

q_in, q_out = queue.Queue(), queue.Queue(maxsize=100)


def worker():
    while True:
        item = q_in.get()
        if item is None:
            return
        i, p = item
        u8 = torch.from_numpy(np.load(p + ".npy")).to(torch.uint8)
        q_out.put((i, (u8 / 255.0).clamp(0.0, 1.0)))


ws = [threading.Thread(target=worker) for _ in range(threads)]
for w in ws:
    w.start()
torch.cuda.synchronize()
t0 = time.perf_counter()
for i, p in enumerate(image_list):
    q_in.put((i, p))
for _ in range(n):
    _, img = q_out.get()
    chw = img.to(dev).permute(2, 0, 1)
torch.cuda.synchronize()
ref = n / (time.perf_counter() - t0)
for _ in ws:
    q_in.put(None)
for w in ws:
    w.join()
print(f"1080p RGB, {n} images, {threads} reader threads: native ring {native:.1f} images/s, "
      f"reference-style threads + float copy {ref:.1f} images/s")
