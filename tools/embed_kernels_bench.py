"""Times the appearance embedding's library kernels at config 2's 1080p shapes (DOGS_HIP_LIB picks the build: run it
once per variant, under rocprofv3 --kernel-trace --stats for the per-kernel split): the fused head forward / backward
(dg_mask_head_*), and dg_conv3x3 (forward, adjoint) and dg_conv3x3_wgrad for every 3x3 convolution of the network
(fusion 67 -> 256 at 34 x 60, the four upsampling stages).  Prints ms per call from events on the library's stream.
python tools/embed_kernels_bench.py [--iters 50] [--miopen]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONVS = [(67, 256, 34, 60), (64, 128, 68, 120), (32, 64, 136, 240), (16, 32, 272, 480), (8, 16, 544, 960)]


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--miopen", action="store_true", help="time MIOpen's forward / backward-data instead")
    args = ap.parse_args()
    from dogs_amd import _lib
    L = _lib.load()
    dev = torch.device("cuda", 0)
    st = _lib.stream_of(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    H, W, h2, w2 = 1080, 1920, 544, 960
    u = torch.rand((16, h2, w2), generator=g, device=dev)
    w1 = torch.randn((8, 16, 3, 3), generator=g, device=dev) * 0.1
    b1 = torch.randn(8, generator=g, device=dev) * 0.1
    w2_ = torch.randn((3, 8, 3, 3), generator=g, device=dev) * 0.1
    b2 = torch.randn(3, generator=g, device=dev) * 0.1
    mask = torch.empty((3, H, W), device=dev)
    dm = torch.randn((3, H, W), generator=g, device=dev)
    du = torch.empty_like(u)
    dp = torch.empty(int(L.dg_mask_head_nparams()), device=dev)
    nb = int(L.dg_mask_head_scratch_bytes(H, W))
    scr = torch.empty(nb, dtype=torch.uint8, device=dev)
    P = [t.data_ptr() for t in (u, w1, b1, w2_, b2)]
    hid = torch.empty((8, H, W), device=dev)
    res = {"head_fwd": timed(lambda: _lib.check(L.dg_mask_head_forward(H, W, h2, w2, *P, mask.data_ptr(),
                                                                       hid.data_ptr(), st)), args.iters),
           "head_bwd": timed(lambda: _lib.check(L.dg_mask_head_backward(H, W, h2, w2, *P, dm.data_ptr(), hid.data_ptr(),
                                                                        du.data_ptr(), dp.data_ptr(), scr.data_ptr(),
                                                                        nb, st)), args.iters),
           "head_bwd_recompute": timed(lambda: _lib.check(L.dg_mask_head_backward(
               H, W, h2, w2, *P, dm.data_ptr(), None, du.data_ptr(), dp.data_ptr(), scr.data_ptr(), nb, st)),
               args.iters)}
    has_conv = hasattr(L, "dg_conv3x3") and not args.miopen
    for cin, cout, h, w in CONVS:
        x = torch.randn((cin, h, w), generator=g, device=dev)
        wt = torch.randn((cout, cin, 3, 3), generator=g, device=dev) * 0.1
        bias = torch.randn(cout, generator=g, device=dev)
        y = torch.empty((cout, h, w), device=dev)
        dy = torch.randn((cout, h, w), generator=g, device=dev)
        dx = torch.empty_like(x)
        dw, db = torch.empty_like(wt), torch.empty_like(bias)
        n = int(L.dg_conv3x3_wgrad_scratch_bytes(cin, cout, h, w))
        s2 = torch.empty(n, dtype=torch.uint8, device=dev)
        key = f"{cin}x{cout}@{h}x{w}"
        if has_conv:
            res["fwd " + key] = timed(lambda: _lib.check(L.dg_conv3x3(cin, cout, h, w, x.data_ptr(), wt.data_ptr(),
                                                                      bias.data_ptr(), y.data_ptr(), 0, None, st)), args.iters)
            res["adj " + key] = timed(lambda: _lib.check(L.dg_conv3x3(cin, cout, h, w, dy.data_ptr(), wt.data_ptr(),
                                                                      None, dx.data_ptr(), 1, None, st)), args.iters)
        else:   # MIOpen's forward and backward-data for comparison
            x4, dy4 = x[None], dy[None]
            res["fwd " + key] = timed(lambda: torch.nn.functional.conv2d(x4, wt, bias, padding=1), args.iters)
            res["adj " + key] = timed(lambda: torch.ops.aten.convolution_backward(
                dy4, x4, wt, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]), args.iters)
        res["wgrad " + key] = timed(lambda: _lib.check(L.dg_conv3x3_wgrad(cin, cout, h, w, x.data_ptr(), dy.data_ptr(),
                                                                          None, 0, dw.data_ptr(), db.data_ptr(),
                                                                          s2.data_ptr(), n, st)), args.iters)
    tot = 0.0
    for k, v in res.items():
        tot += v
        print(f"{k:28s} {v * 1e3:8.1f} us", flush=True)
    print(f"{'total':28s} {tot * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
