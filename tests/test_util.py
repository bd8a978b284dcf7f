"""Image output (mi.util.write_bitmap replacement) and comparison statistics."""
import os

import numpy as np
import pytest


@pytest.mark.parametrize("compression", ["none", "zip", "zips"])
def test_exr_round_trip(tmp_path, compression):
    from mtx import util

    rng = np.random.default_rng(0)
    img = (rng.random((37, 53, 3), dtype=np.float32) * 10).astype(np.float32)
    img[3, 4] = [np.inf, 0.0, -1.5]
    p = os.path.join(tmp_path, "a.exr")
    util.write_exr(p, img, compression)
    back = util.read_exr(p)
    assert back.dtype == np.float32 and back.shape == img.shape
    assert np.array_equal(back, img)
    raw = open(p, "rb").read()
    assert raw[:4] == bytes([0x76, 0x2F, 0x31, 0x01])  # OpenEXR magic
    assert b"channels\0chlist\0" in raw and b"dataWindow\0box2i\0" in raw


def test_exr_zip_compresses_smooth_images(tmp_path):
    from mtx import util

    y, x = np.mgrid[0:64, 0:64].astype(np.float32)
    img = np.stack([x / 64, y / 64, np.zeros_like(x)], -1)
    a, b = os.path.join(tmp_path, "a.exr"), os.path.join(tmp_path, "b.exr")
    util.write_exr(a, img, "none")
    util.write_exr(b, img, "zip")
    assert os.path.getsize(b) < os.path.getsize(a)
    assert np.array_equal(util.read_exr(b), img)


def test_srgb_bitmap_and_stats(tmp_path):
    from mtx import util

    v = util.convert_to_bitmap(np.array([[[0.0, 0.0031308, 1.0]], [[0.5, 2.0, -1.0]]]))
    assert v.dtype == np.uint8 and v[0, 0].tolist() == [0, 10, 255] and v[1, 0].tolist() == [188, 255, 0]
    img = np.full((4, 4, 3), 0.25, np.float32)
    util.write_bitmap(os.path.join(tmp_path, "a.png"), img)
    from PIL import Image

    assert np.asarray(Image.open(os.path.join(tmp_path, "a.png"))).shape == (4, 4, 3)
    ref = np.zeros_like(img)
    assert util.mse(img, ref) == pytest.approx(0.0625) and util.bias(img, ref) == pytest.approx(0.25)
    assert util.variance(img) == 0.0
