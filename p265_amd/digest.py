"""Host restatement of the device picture digest (p265r_batch_digest, csrc/digest.h).

digest(plane) = sum over the plane's 32-bit words (row y, word k, K words per row) of
mix64(word | (y * K + k) << 32) mod 2^64, with mix64 the splitmix64 finalizer and word the
little-endian 32-bit value of the row's bytes 4k..4k+3: samples 4k..4k+3 of a uint8 plane (K = W/4),
samples 2k, 2k+1 of a uint16 plane (BitDepth > 8, K = W/2).  Position-keyed, so a changed, swapped
or shifted sample changes it; a sum, so the device adds partial sums in any order.
"""
import numpy as np

_M1 = np.uint64(0xbf58476d1ce4e5b9)
_M2 = np.uint64(0x94d049bb133111eb)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def plane_digest(plane):
    """Digest of one plane [h][w] (w a multiple of 4) as a Python int: a uint16 plane as 16-bit samples
    (BitDepth > 8), anything else as uint8 samples (8-bit planes; the oracle's integer arrays)."""
    p = np.asarray(plane)
    p = np.ascontiguousarray(p, "<u2" if p.dtype == np.uint16 else np.uint8)
    h, w = p.shape
    if w % 4:
        raise ValueError("plane width %d is not a multiple of 4" % w)
    words = p.view("<u4").astype(np.uint64).ravel()
    pos = np.arange(words.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(_mix64(words | (pos << np.uint64(32))).sum(dtype=np.uint64))


def picture_digest(planes):
    """[Y, Cb, Cr] planes -> uint64 array of 3 digests (p265r_batch_digest's layout)."""
    return np.array([plane_digest(pl) for pl in planes], np.uint64)
