"""GPU tests of the device primitives under the binning: stable radix sort and exclusive scan (bit-exact vs numpy)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sort(keys, vals, b0, b1, dev):
    from dogs_amd import _lib
    k = torch.from_numpy(keys.view(np.int32)).to(dev)
    v = torch.from_numpy(vals.view(np.int32)).to(dev)
    arena = _lib.TensorArena(dev)
    _lib.check(_lib.load().dg_sort_pairs_u32(k.data_ptr(), v.data_ptr(), len(keys), b0, b1, arena.fn, None,
                                             _lib.stream_of(dev)))
    torch.cuda.synchronize()
    return k.cpu().numpy().view(np.uint32), v.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,b1,hi", [(1, 32, 2**32), (100, 8, 256), (4096, 13, 8160), (4097, 32, 2**32),
                                     (100000, 16, 8160), (1 << 20, 32, 1 << 20), (3_000_001, 13, 8160)])
def test_radix_sort_stable(hip_device, n, b1, hi):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    k, v = _sort(keys, vals, 0, b1, hip_device)
    order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(k, keys[order])
    np.testing.assert_array_equal(v, vals[order])


def test_radix_sort_skewed_digits(hip_device):
    # depth-like keys: identical high bytes (all lanes of a wave in one digit group)
    rng = np.random.default_rng(0)
    z = rng.uniform(2.0, 20.0, 500_000).astype(np.float32)
    keys = z.view(np.uint32).copy()
    keys[::7] = 0xFFFFFFFF
    vals = np.arange(keys.size, dtype=np.uint32)
    k, v = _sort(keys, vals, 0, 32, hip_device)
    order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(v, vals[order])


@pytest.mark.parametrize("n", [1, 255, 2048, 2049, 1_000_003])
def test_exclusive_scan(hip_device, n):
    from dogs_amd import _lib
    rng = np.random.default_rng(n)
    x = rng.integers(0, 40, size=n).astype(np.uint32)
    dev = hip_device
    xi = torch.from_numpy(x.view(np.int32)).to(dev)
    out = torch.empty_like(xi)
    tot = torch.zeros(1, dtype=torch.int32, device=dev)
    arena = _lib.TensorArena(dev)
    _lib.check(_lib.load().dg_exclusive_scan_u32(xi.data_ptr(), out.data_ptr(), n, tot.data_ptr(), arena.fn, None,
                                                 _lib.stream_of(dev)))
    torch.cuda.synchronize()
    ref = np.concatenate([[0], np.cumsum(x.astype(np.uint64))[:-1]]).astype(np.uint32)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref)
    assert int(tot.item()) == int(x.astype(np.uint64).sum())
