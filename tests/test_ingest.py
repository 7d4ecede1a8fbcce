"""Ingest (stereo_kitti.py:42-43, cv2.imread(path, cv2.IMREAD_GRAYSCALE)): the native PNG decoder in
liborbfe (host code, no GPU).  Grey images are lossless, so PIL's decode pins them exactly; the colour ->
grey branch follows libpng's rgb_to_gray fixed-point weights, which OpenCV requests — parity unpinned
(OpenCV / libpng headers are absent), checked against a numpy restatement of that formula."""
import io

import numpy as np
import pytest

from conftest import GOLDEN
from pyorbslam_amd import ingest


def _png(arr, mode, **kw):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(arr, mode).save(b, format="PNG", **kw)
    return b.getvalue()


def test_reference_fixture_exact():
    from PIL import Image
    got = ingest.imread(GOLDEN / "kitti06-436.png")
    assert got.dtype == np.uint8 and got.shape == (370, 1226)
    assert np.array_equal(got, np.array(Image.open(GOLDEN / "kitti06-436.png")))


@pytest.mark.parametrize("compress", [0, 1, 6, 9])
def test_grey_and_grey_alpha_exact(compress):
    rng = np.random.default_rng(compress)
    g = (rng.integers(0, 256, (97, 131)) // (1 + compress)).astype(np.uint8)  # mixed filters per row
    g[10:40, 20:90] = np.arange(70, dtype=np.uint8)
    assert np.array_equal(ingest.decode_png(_png(g, "L", compress_level=compress)), g)
    la = np.stack([g, 255 - g], -1)
    assert np.array_equal(ingest.decode_png(_png(la, "LA", compress_level=compress)), g)


@pytest.mark.parametrize("mode", ["RGB", "RGBA"])
def test_colour_to_grey_libpng_weights(mode):
    rng = np.random.default_rng(3)
    c = rng.integers(0, 256, (64, 75, 4 if mode == "RGBA" else 3)).astype(np.uint8)
    r, g, b = (c[..., k].astype(np.int64) for k in range(3))
    want = ((9797 * r + 19234 * g + 3737 * b) >> 15).astype(np.uint8)  # libpng: truncated coefficients and sum
    assert np.array_equal(ingest.decode_png(_png(c, mode)), want)


def test_batch_threads_and_errors(tmp_path):
    rng = np.random.default_rng(9)
    imgs = [rng.integers(0, 256, (40, 52)).astype(np.uint8) for _ in range(9)]
    paths = []
    for i, a in enumerate(imgs):
        p = tmp_path / f"{i:06d}.png"
        p.write_bytes(_png(a, "L"))
        paths.append(str(p))
    for t in (1, 4):
        out = ingest.imread_batch(paths, 52, 40, threads=t)
        assert all(np.array_equal(out[i], imgs[i]) for i in range(9))
    (tmp_path / "bad.png").write_bytes(b"not a png")
    with pytest.raises(RuntimeError, match="EFORMAT"):
        ingest.imread_batch(paths + [str(tmp_path / "bad.png")], 52, 40, threads=3)
    assert ingest.imread(tmp_path / "missing.png") is None
    interlaced = _png(imgs[0], "L", optimize=False)
    assert np.array_equal(ingest.decode_png(interlaced), imgs[0])
