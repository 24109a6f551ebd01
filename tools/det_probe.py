"""Run-to-run determinism of the appearance embedding's backward on the GPU (MIOpen convolutions, the resize adjoint):
the same forward/backward three times from one state, every parameter gradient compared bit for bit; with
torch.backends.cudnn.deterministic off and on."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def grads(net, img, H, W, g):
    net.zero_grad(set_to_none=True)
    m = net(img, 1, (H, W))
    m.backward(g)
    return [p.grad.detach().clone() for p in net.parameters()]


def main():
    from dogs_amd.masks import AppearanceEmbedding
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for H, W in ((120, 160), (300, 400), (1080, 1920)):
        net = AppearanceEmbedding(4).to(dev)
        with torch.no_grad():
            net.appearance_embedding.normal_(0.0, 0.3)
        img = torch.rand((3, (H + 31) // 32, (W + 31) // 32), device=dev)
        g = torch.randn((3, H, W), device=dev)
        for det in (False, True):
            torch.backends.cudnn.deterministic = det
            ref = grads(net, img, H, W, g)
            same = all(all(torch.equal(a, b) for a, b in zip(ref, grads(net, img, H, W, g))) for _ in range(3))
            names = [n for n, _ in net.named_parameters()]
            diff = []
            if not same:
                r2 = grads(net, img, H, W, g)
                diff = [n for n, a, b in zip(names, ref, r2) if not torch.equal(a, b)]
            print(f"{H}x{W} cudnn.deterministic={det}: bitwise repeatable={same} {diff}", flush=True)


if __name__ == "__main__":
    main()
