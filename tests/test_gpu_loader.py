"""GPU parity of the image path: the native pinned ring behind ImageReader and read_image
against oracle/loader_oracle.py (the reference's read_image on the decoded bytes), bit-exact; every submitted image
comes back exactly once (completion order, as the reference's queue)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _write(tmp_path, n, seed):
    rng = np.random.default_rng(seed)
    paths, arrays = [], []
    for i in range(n):
        h, w = int(rng.integers(16, 200)), int(rng.integers(16, 300))
        c = 4 if i % 3 == 2 else 3
        a = rng.integers(0, 256, (h, w, c), dtype=np.uint8)
        p = str(tmp_path / f"img_{i:03d}.png")
        np.save(p + ".npy", a)
        paths.append(p)
        arrays.append(a)
    return paths, arrays


@pytest.mark.parametrize("threads,slots", [(1, 2), (8, 100)])
def test_image_reader_matches_read_image(hip_device, tmp_path, threads, slots):
    from dogs_amd.loader import ImageReader
    from oracle import loader_oracle as L
    paths, arrays = _write(tmp_path, 24, threads)
    rgb = [i for i in range(len(paths)) if arrays[i].shape[2] == 3]
    reader = ImageReader(max_size=slots, max_num_threads=threads, num_channels=3,
                         image_list=[paths[i] for i in rgb], device=hip_device)
    reader.add_task(None)
    seen = []
    for _ in range(len(rgb)):
        k, img = reader.get_image()
        seen.append(k)
        ref = L.read_image(arrays[rgb[k]], 3)
        assert img.shape == ref.shape and img.permute(2, 0, 1).is_contiguous()
        np.testing.assert_array_equal(img.cpu().numpy(), ref)
    assert sorted(seen) == list(range(len(rgb)))
    assert reader.num_images() == 0
    reader.safe_exit()


def test_rgba_reader_and_read_image(hip_device, tmp_path):
    from dogs_amd.loader import ImageReader, read_image
    from oracle import loader_oracle as L
    paths, arrays = _write(tmp_path, 9, 5)
    rgba = [i for i in range(len(paths)) if arrays[i].shape[2] == 4]
    reader = ImageReader(num_channels=4, image_list=[paths[i] for i in rgba], device=hip_device)
    reader.add_task(None)
    for _ in rgba:
        k, img = reader.get_image()
        np.testing.assert_array_equal(img.cpu().numpy(), L.read_image(arrays[rgba[k]], 4))
    reader.safe_exit()
    for i in (0, 2):
        np.testing.assert_array_equal(read_image(paths[i], 4 if arrays[i].shape[2] == 4 else 3,
                                                 device=hip_device).cpu().numpy(),
                                      L.read_image(arrays[i], 4 if arrays[i].shape[2] == 4 else 3))
    torch.cuda.synchronize()
