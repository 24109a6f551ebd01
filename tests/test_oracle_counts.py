"""LightGaussian count mode of the oracle (CountGaussiansCUDA / renderCUDA_count, old_diff-gaussian-rasterization
forward.cu:392-500) against a pure-Python restatement of its per-pixel loop on a tiny scene."""
import math

import numpy as np

from raster_util import oracle_forward, small_scene


def _py_counts(st, P, W, H):
    """Per-pixel front-to-back loop over each tile's sorted list: a Gaussian is counted once per pixel it
    contributes to (accepted, alpha >= 1/255, and not the splat that would drive T below 1e-4)."""
    tiles, idx, _ = st.sorted_list()
    g = st.geom()
    xy, co = g["means2D"], g["conic_opacity"]
    rng = st.ranges()
    count = np.zeros(P, np.int64)
    score = np.zeros(P, np.float64)
    tx = (W + 15) // 16
    for t in range(len(rng)):
        r0, r1 = int(rng[t][0]), int(rng[t][1])
        x0, y0 = (t % tx) * 16, (t // tx) * 16
        for py in range(y0, min(y0 + 16, H)):
            for px in range(x0, min(x0 + 16, W)):
                T = 1.0
                for j in range(r0, r1):
                    gi = int(idx[j])
                    dx, dy = xy[gi, 0] - px, xy[gi, 1] - py
                    a, b, c, o = (float(v) for v in co[gi])
                    power = -0.5 * (a * dx * dx + c * dy * dy) - b * dx * dy
                    if power > 0.0:
                        continue
                    alpha = min(0.99, o * math.exp(power))
                    if alpha < 1.0 / 255.0:
                        continue
                    test_T = T * (1.0 - alpha)
                    if test_T < 0.0001:
                        break
                    count[gi] += 1
                    score[gi] += o
                    T = test_T
    return count, score


def test_oracle_counts_match_python_loop(oracle):
    W, H, n = 40, 24, 60
    s = small_scene(n, W, H, seed=9)
    _, radii, _, st = oracle_forward(oracle, s, (0.0, 0.0, 0.0))
    cnt, score = st.counts()
    cnt_py, score_py = _py_counts(st, n, W, H)
    assert cnt.sum() > 0
    assert np.all(cnt[radii == 0] == 0)
    # float32 (oracle) vs float64 (here) may flip a decision right at a threshold; allow one pixel
    assert np.abs(cnt - cnt_py).max() <= 1
    assert (cnt == cnt_py).mean() > 0.95
    np.testing.assert_allclose(score[cnt == cnt_py], score_py[cnt == cnt_py], rtol=1e-5)
