"""The packed level keys of round 6 ((x + y * w) | score << 24, orbfe_common.h kKeyXYBits) are decoded in the
kernels as y = mul_hi(xy, mag) >> sh, x = xy - y * w with mag = ceil(2^(31 + s) / w), sh = s - 1,
s = ceil(log2 w) (orbfe_host.hip key_divisor, orbfe_kernels.hip key_xy).  This pins that arithmetic on the
CPU for every level width the library accepts (2 .. 32 767): exact floor division for the indices where the
error term is largest (the last rows below 2^24) and at every row boundary of the first rows."""
import numpy as np


def magic(w: int) -> tuple[int, int]:
    s = (w - 1).bit_length()
    return -(-(1 << (31 + s)) // w), s - 1


def test_key_divisor_exact_for_every_width():
    bad = []
    for w in range(2, 32768):
        mag, sh = magic(w)
        assert mag < 2 ** 32, w
        h = (1 << 24) // w
        ys = np.unique(np.concatenate([np.arange(0, min(h, 8)), np.arange(max(h - 8, 0), h)])).astype(np.uint64)
        xy = np.concatenate([ys * np.uint64(w), ys * np.uint64(w) + np.uint64(w - 1)])
        xy = xy[xy < (1 << 24)]
        q = ((xy * np.uint64(mag)) >> np.uint64(32)) >> np.uint64(sh)
        x = xy - q * np.uint64(w)
        if not (np.array_equal(q, xy // np.uint64(w)) and (x < w).all()):
            bad.append(w)
    assert not bad, bad[:10]


def test_key_divisor_exhaustive_for_a_kitti_level():
    """Every index of a 1 241 x 376 level (KITTI level 0) and of a 4 500 x 600 one."""
    for w, h in ((1241, 376), (4500, 600), (2500, 4500)):
        mag, sh = magic(w)
        xy = np.arange(w * h, dtype=np.uint64)
        q = ((xy * np.uint64(mag)) >> np.uint64(32)) >> np.uint64(sh)
        assert np.array_equal(q, xy // np.uint64(w))
