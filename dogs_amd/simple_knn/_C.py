"""simple_knn._C.distCUDA2 (reference simple-knn/spatial.cu:18-35) over libdogs_hip.so."""
from __future__ import annotations

import torch

from .. import _lib


def distCUDA2(points: torch.Tensor) -> torch.Tensor:  # noqa: N802
    """Mean squared distance of each point to its 3 (approximate, Morton-box) nearest neighbours."""
    _lib.require_device(points, "points")
    p = points.contiguous() if points.dtype == torch.float32 else points.float().contiguous()
    P = int(p.size(0))
    out = torch.zeros((P,), dtype=torch.float32, device=p.device)
    if P == 0:
        return out
    with _lib.device_ctx(p.device):
        arena = _lib.TensorArena(p.device)
        _lib.check(_lib.load().dg_dist_cuda2(P, p.data_ptr(), out.data_ptr(), arena.fn, None,
                                             _lib.stream_of(p.device)))
    return out
