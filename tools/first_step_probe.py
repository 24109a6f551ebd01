"""Native vs autograd first training step (tests/test_gpu_trainer_options.py::test_first_step_native_equals_autograd):
per-group relative differences of the first Adam moments (all rows, and without the degenerate row) for the plain,
zero-scaling and antialiasing cases."""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from test_gpu_trainer import _cfg, _normal, _problem
    from test_gpu_trainer_options import _rel, _state
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = torch.device("cuda", 0)
    import dogs_amd.gaussian_model as GM
    from dogs_amd.activations import activate
    torch_props = {k: getattr(GM.GaussianSplatModel, k) for k in ("get_opacity", "get_scaling", "get_quaternion")}

    def ours(kind):   # the model's activations through the library's kernels (the native step's expressions)
        def get(self):
            o, s, q = activate(self._opacity, self._scaling, self._quaternion)
            return {"get_opacity": o, "get_scaling": s, "get_quaternion": q}[kind]
        return property(get)
    for case in ("plain", "plain-kernel-activations", "zero-scaling", "antialiasing"):
        for k, v in torch_props.items():
            setattr(GM.GaussianSplatModel, k, ours(k) if case.endswith("kernel-activations") else v)
        kw = dict(densify_start_iter=10 ** 6, opacity_reset_interval=10 ** 6, prune_iterations=(),
                  lambda_scale=0.05)
        if case == "antialiasing":
            kw.update(anti_aliasing=True)
        cfg = _cfg(**kw)
        out = []
        for native in (True, False):
            m, cams, gts = _problem(dev, n_true=30_000, n_init=6_000, W=400, H=300, views=2)
            m.active_sh_degree = 3
            with torch.no_grad():
                gen = torch.Generator(device=dev).manual_seed(4)
                m._features_rest.normal_(0.0, 0.05, generator=gen)
                m._scaling.add_(torch.randn(m._scaling.shape, generator=gen, device=dev) * 0.3)
                m._quaternion.add_(torch.randn(m._quaternion.shape, generator=gen, device=dev) * 0.3)
                if case.startswith("zero"):
                    m._scaling[7, 1] = -200.0
            tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=2, native=native, normal=_normal(dev, 3))
            tr.train_iteration()
            tr.sync()
            out.append(_state(tr))
        s0, s1 = out
        rows = torch.ones(s0[0]["xyz"].shape[0], dtype=torch.bool, device=dev)
        rows[7] = False
        msg = []
        for k in s0[1]:
            a, b = s0[1][k][0], s1[1][k][0]
            d = (a - b).abs().amax(dim=tuple(range(1, a.dim())))
            msg.append(f"{k}: all {_rel(a, b):.2e} ex7 {_rel(a[rows], b[rows]):.2e} worst row {int(d.argmax())}")
        print(case, "; ".join(msg), flush=True)


if __name__ == "__main__":
    main()
