"""Image writers of the drop-in (gi_write_image = R2Image::Write, R2Image.cpp:316-339), CPU only.

JPEG: the reference writes through its vendored IJG libjpeg (quality 75, optimize_coding,
JDCT_ISLOW, jpeg_set_defaults: JFIF 1.01, YCbCr 4:2:0; R2Image.cpp:1094-1163). The same library
algorithms are in the image's PIL (libjpeg), so PIL's encoding of the same pixels with those
settings is the pin: the files must be byte-identical (odd sizes exercise the edge padding and
libjpeg's dummy blocks). The other formats are checked field by field against the reference
writers' layouts.
"""
import io
import struct

import numpy as np
import pytest

import gi_amd

PIL = pytest.importorskip("PIL.Image")


def _image(w, h, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    img = np.stack([x * 255.0 / max(1, w - 1), y * 255.0 / max(1, h - 1), (x + y) * 3.0 % 256], -1)
    return np.clip(img + rng.normal(0, 20, img.shape), 0, 255).astype(np.uint8)  # rows bottom-up


@pytest.mark.parametrize("w,h", [(64, 48), (37, 29), (17, 9), (1, 1), (16, 17), (200, 133)])
def test_jpeg_bytes_equal_libjpeg(tmp_path, w, h):
    img = _image(w, h, seed=w * h)
    path = str(tmp_path / "a.jpg")
    gi_amd.write_image(path, img)
    ours = open(path, "rb").read()
    b = io.BytesIO()
    PIL.fromarray(img[::-1]).save(b, format="JPEG", quality=75, optimize=True, subsampling=2)
    assert ours == b.getvalue()
    gi_amd.write_image(str(tmp_path / "a.jpeg"), img)
    assert open(str(tmp_path / "a.jpeg"), "rb").read() == ours


def test_bmp_layout(tmp_path):
    img = _image(13, 7)  # 39-byte rows: 1 byte of padding each
    path = str(tmp_path / "a.bmp")
    gi_amd.write_image(path, img)
    d = open(path, "rb").read()
    assert d[:2] == b"BM"
    size, _, _, off = struct.unpack("<IHHI", d[2:14])
    bi = struct.unpack("<IiiHHIIiiII", d[14:54])
    assert off == 54 and size == 54 + 40 * 7 and bi[:5] == (40, 13, 7, 1, 24)
    assert bi[5] == 0 and bi[6] == 40 * 7 and bi[7] == bi[8] == 2925
    rows = np.frombuffer(d[54:], dtype=np.uint8).reshape(7, 40)[:, :39].reshape(7, 13, 3)
    np.testing.assert_array_equal(rows[..., ::-1], img)  # bottom-up rows, BGR
    np.testing.assert_array_equal(np.asarray(PIL.open(path).convert("RGB")), img[::-1])


def test_ppm_ascii_layout(tmp_path):
    img = _image(6, 3)
    path = str(tmp_path / "a.ppm")
    gi_amd.write_image(path, img)
    lines = open(path).read().split("\n")
    assert lines[:3] == ["P3", "6 3", "255"]
    # four pixels per line, "%-3d %-3d %-3d  " each; a short last line per row (6 % 4 != 0)
    px = img[2, 0]
    assert lines[3].startswith("%-3d %-3d %-3d  " % tuple(px))
    vals = np.array(open(path).read().split()[4:], dtype=int).reshape(3, 6, 3)
    np.testing.assert_array_equal(vals, img[::-1])
    assert len(lines) == 3 + 3 * 2 + 2


def test_pgm_binary_gray(tmp_path):
    img = _image(5, 4)
    path = str(tmp_path / "a.pgm")
    gi_amd.write_image(path, img)
    d = open(path, "rb").read()
    assert d.startswith(b"P5\n5 4\n255\n")
    g = np.frombuffer(d[len(b"P5\n5 4\n255\n"):], dtype=np.uint8).reshape(4, 5)
    top = img[::-1].astype(float)
    want = (0.30 * top[..., 0] + 0.59 * top[..., 1] + 0.11 * top[..., 2]).astype(int)
    np.testing.assert_array_equal(g, want)


def test_raw_planar_floats(tmp_path):
    img = _image(4, 3)
    path = str(tmp_path / "a.raw")
    gi_amd.write_image(path, img)
    d = open(path, "rb").read()
    assert struct.unpack("<4I", d[:16]) == (54321, 4, 3, 3)
    f = np.frombuffer(d[16:], dtype=np.float32).reshape(3, 3, 4)  # [component][row][col]
    np.testing.assert_array_equal(f, np.moveaxis(img, -1, 0) / np.float32(255.0))


def test_tiff_unsupported_like_the_reference(tmp_path):
    """R2Image::WriteTIFF without RN_USE_TIFF (the reference's build): "TIFF not supported"."""
    with pytest.raises(gi_amd.GiError):
        gi_amd.write_image(str(tmp_path / "a.tif"), _image(4, 4))
    with pytest.raises(gi_amd.GiError):
        gi_amd.write_image(str(tmp_path / "a.gif"), _image(4, 4))
