"""The OpenMP oracle gives bit-identical results for any thread count (gs_oracle.c header): sorted instance list,
ranges, radii, images, per-pixel state, count-mode counts and scores, and all backward outputs.  This is what lets
the full-size GPU parity tests and the bench's all-core CPU baseline use every host core."""
import numpy as np

from raster_util import oracle_forward, small_scene


def _run(O, s, W, H, threads):
    old = O.set_threads(threads)
    try:
        col, radii, inv, st = oracle_forward(O, s, (0.1, 0.2, 0.3))
        rng = np.random.default_rng(4)
        g = st.backward(rng.standard_normal((3, H, W)).astype(np.float32),
                        (0.1 * rng.standard_normal((H, W))).astype(np.float32))
        return dict(col=col, radii=radii, inv=inv, lst=st.sorted_list(), ranges=st.ranges(),
                    img=st.image_state(), counts=st.counts(), g=g)
    finally:
        O.set_threads(old)


def test_oracle_thread_count_invariance(oracle):
    n, W, H = 6000, 333, 211
    s = small_scene(n, W, H, seed=17)
    a = _run(oracle, s, W, H, 1)
    b = _run(oracle, s, W, H, 7)
    for k in ("col", "radii", "inv", "ranges"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for x, y in zip(a["lst"] + a["img"] + a["counts"], b["lst"] + b["img"] + b["counts"]):
        np.testing.assert_array_equal(x, y)
    assert int(a["counts"][0].sum()) > 0
    for k, v in a["g"].items():
        np.testing.assert_array_equal(v, b["g"][k], err_msg=k)
