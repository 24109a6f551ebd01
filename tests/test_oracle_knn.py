"""simple-knn's distCUDA2 (simple_knn.cu:147-183) is an exact search: the +-3 Morton neighbours only bound the box
pruning (a box farther than the current 3rd-best cannot hold a nearer point), so the result is the mean of the three
smallest squared distances to the other points.  The oracle's restatement is checked here against a brute-force
search with the reference's float32 arithmetic as nvcc compiles it -- the squared distance contracted into fused
multiply-adds, fma(dz, dz, fma(dy, dy, dx dx)) (nvcc's default --fmad=true; the oracle and the HIP kernel spell the
fmas out), the three best ascending, ((b0 + b1) + b2) / 3 -- bit for bit, on uniform, clustered and duplicated point
sets.  The fma is emulated exactly: a product of two float32 values is exact in float64, and the float64 sum is
rounded once to float32 (a double rounding could differ from a true fma only for sums needing more than 53 bits, which
these magnitudes do not).  CPU only."""
import numpy as np
import pytest


def brute_knn_mean3(p):
    p = np.asarray(p, np.float32)
    out = np.empty(p.shape[0], np.float32)
    for i0 in range(0, p.shape[0], 512):
        q = p[i0:i0 + 512]
        d = (p[None, :, :] - q[:, None, :]).astype(np.float64)  # point - ref, the difference rounded in float32
        t = (d[..., 0] * d[..., 0]).astype(np.float32).astype(np.float64)
        t = (d[..., 1] * d[..., 1] + t).astype(np.float32).astype(np.float64)
        d2 = (d[..., 2] * d[..., 2] + t).astype(np.float32)
        d2[np.arange(q.shape[0]), np.arange(i0, i0 + q.shape[0])] = np.inf      # not itself (by index)
        b = np.sort(np.partition(d2, 2, axis=1)[:, :3], axis=1)
        out[i0:i0 + 512] = ((b[:, 0] + b[:, 1]) + b[:, 2]) / np.float32(3.0)
    return out


@pytest.mark.parametrize("kind,P", [("uniform", 3000), ("clustered", 2500), ("duplicates", 1200), ("tiny", 5)])
def test_oracle_knn_matches_brute_force(oracle, kind, P):
    rng = np.random.default_rng(P)
    if kind == "uniform":
        p = rng.uniform(-5, 5, (P, 3))
    elif kind == "clustered":
        c = rng.uniform(-20, 20, (25, 3))
        p = c[rng.integers(0, 25, P)] + 0.05 * rng.standard_normal((P, 3))
    elif kind == "duplicates":
        base = rng.uniform(-1, 1, (P // 3, 3))
        p = np.concatenate([base, base, base + 1e-3])
    else:
        p = rng.uniform(-1, 1, (P, 3))
    p = p.astype(np.float32)
    got = oracle.knn_dist2(p)
    np.testing.assert_array_equal(got, brute_knn_mean3(p))
