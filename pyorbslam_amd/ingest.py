"""Image ingest of the front-end: cv2.imread(path, cv2.IMREAD_GRAYSCALE) as the reference's driver calls it
(stereo_kitti.py:42-43), decoded natively in liborbfe (orbfe_png_decode / orbfe_png_read_batch: zlib
inflate + PNG row unfiltering, colour to grey with libpng's rgb_to_gray weights).  imread_batch decodes a
list of same-size files with a pool of host threads into one array (the batched-frames mode's staging
before a single host-to-device copy)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import call, ptr

IMREAD_GRAYSCALE = 0  # cv2.IMREAD_GRAYSCALE


def decode_png(data: bytes | np.ndarray) -> np.ndarray:
    buf = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, np.uint8)
    w, h = C.c_int32(), C.c_int32()
    call("orbfe_png_decode", ptr(buf), buf.size, None, 0, C.byref(w), C.byref(h))
    out = np.empty((h.value, w.value), np.uint8)
    call("orbfe_png_decode", ptr(buf), buf.size, ptr(out), w.value, C.byref(w), C.byref(h))
    return out


def imread(path, flags: int = IMREAD_GRAYSCALE):
    """cv2.imread for PNG files as grey images; like cv2.imread, None when the file cannot be read."""
    if flags != IMREAD_GRAYSCALE:
        raise ValueError("only cv2.IMREAD_GRAYSCALE (the reference's flag) is supported")
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    return decode_png(data)


def imread_batch(paths, width: int, height: int, threads: int | None = None, out: np.ndarray | None = None) -> np.ndarray:
    """(n, height, width) uint8 from n same-size PNG files, decoded by `threads` host threads."""
    n = len(paths)
    if out is None:
        out = np.empty((n, height, width), np.uint8)
    if out.shape != (n, height, width) or out.dtype != np.uint8 or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous (n, height, width) uint8 array")
    if threads is None:
        try:
            threads = min(16, len(os.sched_getaffinity(0)))
        except AttributeError:  # pragma: no cover
            threads = 4
    arr = (C.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    call("orbfe_png_read_batch", arr, n, width, height, ptr(out), int(threads))
    return out
