"""Known answers of the read_image restatement (oracle/loader_oracle.py, task_queue.py:13-27)."""
import numpy as np

from oracle import loader_oracle as L


def test_read_image_rgb_and_rgba():
    u8 = np.array([[[0, 255, 51], [102, 204, 1]]], np.uint8)
    img = L.read_image(u8, 3)
    assert img.dtype == np.float32 and img.shape == (1, 2, 3)
    np.testing.assert_array_equal(img[0, 0], np.array([0, 1, 0.2], np.float32))
    rgba = np.array([[[255, 255, 255, 0], [255, 0, 128, 255]]], np.uint8)
    out = L.read_image(rgba, 4)
    assert out.shape == (1, 2, 3)
    np.testing.assert_array_equal(out[0, 0], 0)            # fully transparent over black
    np.testing.assert_array_equal(out[0, 1], np.array([1, 0, np.float32(128) / np.float32(255)], np.float32))
