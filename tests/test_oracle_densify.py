"""Known-answer checks of the densification restatement (oracle/densify_oracle.py): row order, optimizer-state
handling and the prune rules of gaussian_splat_model.py:434-531 on hand-built cases (the reference ships no fixture
for these functions: parity of the restatement itself is unpinned)."""
import numpy as np

from oracle import densify_oracle as D


def _model(n):
    rng = np.random.default_rng(0)
    p = {"xyz": rng.standard_normal((n, 3)).astype(np.float32),
         "f_dc": rng.standard_normal((n, 1, 3)).astype(np.float32),
         "f_rest": rng.standard_normal((n, 15, 3)).astype(np.float32),
         "opacity": np.full((n, 1), 2.0, np.float32),
         "scaling": np.full((n, 3), np.log(0.005), np.float32),
         "quaternion": np.tile(np.array([[1, 0, 0, 0]], np.float32), (n, 1))}
    m = {k: (np.full_like(v, 0.5), np.full_like(v, 0.25)) for k, v in p.items()}
    return p, m


def test_clone_split_prune_order():
    p, m = _model(4)
    # 0: large gradient, small -> clone; 1: large gradient, large -> split; 2: transparent -> pruned; 3: kept
    p["scaling"][1] = np.log(0.5)
    p["opacity"][2] = -10.0
    acc = np.array([[1.0], [1.0], [0.0], [0.0]], np.float32)
    den = np.array([[1.0], [1.0], [1.0], [0.0]], np.float32)   # 0/0 -> NaN -> 0
    samples = np.array([[0.1, 0.0, 0.0], [0.0, -0.1, 0.0]], np.float32)
    out, mom, st = D.densify_and_prune(p, m, acc, den, np.zeros(4, np.float32), 2e-4, 0.005, 1.0, None, 0.01,
                                       samples)
    # [originals not split and not pruned: 0, 3] + [clone of 0] + [children of 1 (replica 0, replica 1)]
    np.testing.assert_array_equal(out["f_dc"], np.stack([p["f_dc"][i] for i in (0, 3, 0, 1, 1)]))
    np.testing.assert_allclose(out["xyz"][3], p["xyz"][1] + samples[0], rtol=1e-6)
    np.testing.assert_allclose(out["xyz"][4], p["xyz"][1] + samples[1], rtol=1e-6)
    np.testing.assert_allclose(np.exp(out["scaling"][3]), 0.5 / 1.6, rtol=1e-6)
    # originals keep their moments, appended rows start from zero
    np.testing.assert_array_equal(mom["xyz"][0][:2], 0.5)
    np.testing.assert_array_equal(mom["xyz"][0][2:], 0.0)
    assert all(v.shape[0] == 5 and not v.any() for v in st.values())


def test_size_prune_uses_reset_screen_radii():
    """max_radii2D is reset by densification_postfix before the prune, so only the world-space size prunes."""
    p, m = _model(3)
    p["scaling"][2] = np.log(0.2)   # > 0.1 * extent
    z = np.zeros((3, 1), np.float32)
    out, _, _ = D.densify_and_prune(p, m, z, z + 1, np.full(3, 1e6, np.float32), 1.0, 0.005, 1.0, 20.0, 0.01,
                                    np.zeros((0, 3), np.float32))
    assert out["xyz"].shape[0] == 2


def test_densification_stats():
    mr = np.array([1.0, 5.0, 0.0], np.float32)
    acc = np.zeros((3, 1), np.float32)
    den = np.zeros((3, 1), np.float32)
    g = np.array([[3.0, 4.0, 9.0], [1.0, 0.0, 0.0], [6.0, 8.0, 0.0]], np.float32)
    D.densification_stats(mr, acc, den, np.array([4, 2, 7], np.int32), g, np.array([True, True, False]))
    np.testing.assert_array_equal(mr, [4.0, 5.0, 0.0])
    np.testing.assert_array_equal(acc[:, 0], [5.0, 1.0, 0.0])
    np.testing.assert_array_equal(den[:, 0], [1.0, 1.0, 0.0])
