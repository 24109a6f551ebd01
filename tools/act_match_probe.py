"""How the library's activation kernels (dg_activate_forward: the native step's expressions) compare with torch's
sigmoid / exp / F.normalize (the reference model's get_opacity / get_scaling / get_quaternion) on random inputs, and
which float32 evaluation orders of the quaternion norm reproduce torch's bit for bit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def frac_diff(a, b):
    return float((a != b).float().mean())


def main():
    from dogs_amd.activations import activate
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    n = 1 << 20
    ro = torch.randn((n, 1), generator=g, device=dev) * 3
    rs = torch.randn((n, 3), generator=g, device=dev) * 2 - 4
    rq = torch.randn((n, 4), generator=g, device=dev)
    o, s, q = activate(ro, rs, rq)
    print("sigmoid mismatch", frac_diff(o, torch.sigmoid(ro)))
    print("exp mismatch", frac_diff(s, torch.exp(rs)))
    tq = torch.nn.functional.normalize(rq)
    print("normalize mismatch", frac_diff(q, tq))
    x0, x1, x2, x3 = rq.unbind(1)
    cands = {
        "((x0x0+x1x1)+x2x2)+x3x3": ((x0 * x0 + x1 * x1) + x2 * x2) + x3 * x3,
        "(x0x0+x1x1)+(x2x2+x3x3)": (x0 * x0 + x1 * x1) + (x2 * x2 + x3 * x3),
        "(x0x0+x2x2)+(x1x1+x3x3)": (x0 * x0 + x2 * x2) + (x1 * x1 + x3 * x3),
        "sum(dim=1)": (rq * rq).sum(1),
        "linalg.vector_norm^2": torch.linalg.vector_norm(rq, dim=1) ** 2,
    }
    tn = torch.linalg.vector_norm(rq, dim=1, keepdim=True)
    print("F.normalize == x / vector_norm.clamp_min(eps):", frac_diff(tq, rq / tn.clamp_min(1e-12)))
    for k, ss in cands.items():
        nn = torch.sqrt(ss).unsqueeze(1)
        print(f"norm {k}: norm mismatch {frac_diff(nn, tn):.4f}, q mismatch {frac_diff(rq / nn.clamp_min(1e-12), tq):.4f}")
    # the hypot / fma chain variants
    import math
    fm = torch.sqrt(torch.addcmul(torch.addcmul(torch.addcmul(x0 * x0, x1, x1), x2, x2), x3, x3)).unsqueeze(1)
    print(f"norm fma chain: norm mismatch {frac_diff(fm, tn):.4f}")


if __name__ == "__main__":
    main()
