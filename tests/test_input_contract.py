"""The input contract of the pyORBExtractor drop-in, pinned to the reference caster
(opencv_type_casters.h:163-200): cv::Mat(nh, nw, CV_8UC1, info.ptr) from the buffer's first element with
numpy's strides ignored, uint8 only here (int32 / float32 are undefined behaviour downstream of the
reference's caster and raise), 2-D or single-channel 3-D."""
import numpy as np
import pytest

from pyorbslam_amd.pyORBExtractor import as_gray_u8


def _img():
    return (np.arange(376 * 1241, dtype=np.int64) * 7 % 251).astype(np.uint8).reshape(376, 1241)


def test_contiguous_is_passed_through():
    a = _img()
    assert as_gray_u8(a) is a or np.shares_memory(as_gray_u8(a), a)


@pytest.mark.parametrize("view", ["roi", "rows2", "cols_tail", "chan3d", "transposed"])
def test_strided_views_read_consecutive_bytes_from_the_first_element(view):
    a = _img()
    v = {"roi": a[40:300, 100:600], "rows2": a[::2], "cols_tail": a[:, 700:],
         "chan3d": a[:, :, None][:, 3:900], "transposed": a.T}[view]
    nh, nw = v.shape[:2]
    first = v.__array_interface__["data"][0] - a.__array_interface__["data"][0]
    want = a.reshape(-1)[first:first + nh * nw].reshape(nh, nw)
    got = as_gray_u8(v)
    assert got.shape == (nh, nw) and np.array_equal(got, want) and np.shares_memory(got, a)
    assert not np.array_equal(got, np.ascontiguousarray(v.reshape(nh, nw)))  # not the pixels the view shows


def test_reads_past_the_buffer_raise():
    a = _img()
    with pytest.raises(RuntimeError, match="past its buffer"):
        as_gray_u8(a[::-1])   # first element = last row: the reference reads out of bounds
    with pytest.raises(RuntimeError, match="past its buffer"):
        as_gray_u8(a[:, ::-1])  # first element = the first row's last byte


@pytest.mark.parametrize("dtype", [np.int32, np.float32, np.float64, np.uint16, np.int8])
def test_other_dtypes_raise(dtype):
    with pytest.raises(RuntimeError, match="Unsupported type"):
        as_gray_u8(np.zeros((40, 40), dtype))


def test_dims_and_channels():
    with pytest.raises(RuntimeError, match="Unsupported dim"):
        as_gray_u8(np.zeros((4,), np.uint8))
    with pytest.raises(RuntimeError, match="multi-channel"):
        as_gray_u8(np.zeros((40, 40, 3), np.uint8))
    assert as_gray_u8(np.zeros((40, 40, 1), np.uint8)).shape == (40, 40)


def test_keypoint_tuples_equal_structured_tolist():
    """keypoint_tuples builds the caster's tuples from per-field lists: the same values and element types as
    the structured array's tolist (Python floats, an int octave)."""
    from pyorbslam_amd._lib import KP_DTYPE
    from pyorbslam_amd.pyORBExtractor import keypoint_tuples
    rng = np.random.default_rng(0)
    a = np.zeros(257, KP_DTYPE)
    for f in ("x", "y", "size", "angle", "response"):
        a[f] = rng.random(257).astype(np.float32) * 1000
    a["octave"] = rng.integers(0, 8, 257)
    got, ref = keypoint_tuples(a), a.tolist()
    assert got == ref and [tuple(map(type, t)) for t in got] == [tuple(map(type, t)) for t in ref]
    assert keypoint_tuples(a[:0]) == []
