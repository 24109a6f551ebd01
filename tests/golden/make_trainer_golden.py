"""Generate the trainer-option fixtures under tests/golden/ (run in the build container, never on the GPU box).

    python tests/golden/make_trainer_golden.py

  appearance_embedding.npz  the reference's own AppearanceEmbedding (conerf/model/gaussian_fields/masks.py:8-54,
                            imported by file path from /root/reference) with every parameter set by `fill` below
                            (a formula of its state-dict key and shape, so no weights are stored): the state-dict
                            keys and shapes, a seeded 3 x 4 x 5 input (the 32x-downsampled target of a 100 x 130
                            view) and the [3, 100, 130] mask it returns for view index 2
  reference_configs.json    the trainer keys of the reference configs GSTrainConfig / ADMMRunConfig.from_reference
                            read (urban3d_admm.yaml, mipnerf360.yaml), as parsed values: data for the key-by-key test
                            when /root/reference is absent
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def fill(key: str, shape) -> torch.Tensor:
    """Deterministic parameter values from the key and shape only."""
    n = int(np.prod(shape)) if len(shape) else 1
    h = sum(ord(c) for c in key) % 97
    x = torch.arange(n, dtype=torch.float64)
    v = 0.05 * torch.sin(0.37 * x + h) + 0.01 * torch.cos(0.011 * x * (1 + h % 5))
    return v.reshape(shape).to(torch.float32)


def make_embedding():
    spec = importlib.util.spec_from_file_location("ref_masks", os.path.join(REF, "conerf/model/gaussian_fields/masks.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    net = mod.AppearanceEmbedding(5)
    sd = net.state_dict()
    net.load_state_dict({k: fill(k, tuple(v.shape)) for k, v in sd.items()})
    g = torch.Generator().manual_seed(4)
    img = torch.rand((3, 4, 5), generator=g)
    with torch.no_grad():
        out = net(img, 2, (100, 130))
    keys = sorted(sd)
    np.savez_compressed(os.path.join(HERE, "appearance_embedding.npz"), image=img.numpy(), out=out.numpy(),
                        keys=np.array(keys), shapes=np.array([json.dumps(list(sd[k].shape)) for k in keys]))


def make_configs():
    out = {}
    for name in ("urban3d_admm.yaml", "mipnerf360.yaml"):
        with open(os.path.join(REF, "config/gaussian_splatting", name), encoding="utf-8") as f:
            d = yaml.safe_load(f)
        out[name] = {k: d[k] for k in ("trainer", "prune", "optimizer", "geometry", "texture", "appearance", "loss",
                                       "dataset") if k in d}
        out[name]["dataset"] = {"apply_mask": d["dataset"].get("apply_mask", False)}
    with open(os.path.join(HERE, "reference_configs.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    torch.set_num_threads(1)
    make_embedding()
    make_configs()
    print("ok")
