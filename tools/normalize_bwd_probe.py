"""Which elementwise expression is torch's F.normalize backward on the GPU, bit for bit?  Candidates are evaluated
with eager torch ops (one rounding per op, no contraction) against autograd over 1e6 random quaternions (plus rows
with a zero component and near-degenerate norms).  python tools/normalize_bwd_probe.py"""
import torch
import torch.nn.functional as F


def main():
    dev = torch.device("cuda", 0)
    g0 = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn((1 << 20, 4), generator=g0, device=dev) * torch.rand((1 << 20, 1), generator=g0, device=dev) * 3
    x[:1000, 2] = 0.0
    g = torch.randn(x.shape, generator=g0, device=dev)
    xr = x.clone().requires_grad_(True)
    F.normalize(xr, dim=-1).backward(g)
    ref = xr.grad
    n = ((x[:, 0:1] * x[:, 0:1] + x[:, 1:2] * x[:, 1:2]) + (x[:, 2:3] * x[:, 2:3] + x[:, 3:4] * x[:, 3:4]))
    n = n.sqrt()
    assert torch.equal(n, torch.linalg.vector_norm(x, dim=-1, keepdim=True)), "norm association"
    t1 = -g * ((x / n) / n)
    t2 = -(g * x) / (n * n)
    t3 = (-g * x) / n / n
    sums = {
        "seq": lambda t: ((t[:, 0:1] + t[:, 1:2]) + t[:, 2:3]) + t[:, 3:4],
        "pair": lambda t: (t[:, 0:1] + t[:, 1:2]) + (t[:, 2:3] + t[:, 3:4]),
        "pair02": lambda t: (t[:, 0:1] + t[:, 2:3]) + (t[:, 1:2] + t[:, 3:4]),
        "torchsum": lambda t: t.sum(dim=1, keepdim=True),
    }
    res = {}
    for tn, t in (("t=-g*((x/n)/n)", t1), ("t=-(g*x)/(n*n)", t2), ("t=((-g*x)/n)/n", t3)):
        for sn, f in sums.items():
            s = f(t)
            for bn, b in (("s*(x/n)", s * (x / n)), ("x*(s/n)", x * (s / n)), ("(s*x)/n", (s * x) / n),
                          ("(x/n)*s", (x / n) * s)):
                for an, a in (("g/n+b", g / n + b), ("b+g/n", b + g / n)):
                    got = a
                    key = f"{tn} sum={sn} b={bn} {an}"
                    res[key] = int((got != ref).sum())
    for k, v in sorted(res.items(), key=lambda kv: kv[1])[:12]:
        print(f"{v:9d} mismatches  {k}")
    print("rows:", x.shape[0] * 4, "elements")


if __name__ == "__main__":
    main()
