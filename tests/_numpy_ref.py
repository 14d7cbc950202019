"""Independent numpy restatement of the synthetic plane generators.

Written separately from oracle/pbx_oracle.c and csrc/pbx_common.h so that the three agree
only if each follows the definitions: G_FAKE = Bio-Formats FakeReader.openBytes
(pixel = typeMin + x, 10-pixel boxes {series, planeNo, z, c, t} on rows y < 10);
G_NOISE = splitmix64 counter-hash noise, 257..1486.
"""
import numpy as np

DTYPES_BE = [">i1", ">u1", ">i2", ">u2", ">i4", ">u4", ">f4", ">f8"]
TYPE_MIN = [-128, 0, -32768, 0, -(1 << 31), 0, 0, 0]


def _splitmix(k):
    with np.errstate(over="ignore"):
        z = k + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _cast(pt, v):
    v = np.asarray(v, dtype=np.int64)
    if pt <= 5:
        bits = [8, 8, 16, 16, 32, 32][pt]
        u = (v & ((1 << bits) - 1)).astype(np.uint64)
        return u.astype(DTYPES_BE[pt].replace(">i", ">u"), copy=False).view(DTYPES_BE[pt]) \
            if pt in (0, 2, 4) else u.astype(DTYPES_BE[pt])
    return v.astype(DTYPES_BE[pt])


def region(kind, pt, x0, y0, w, h, seed=0, plane_no=0, z=0, c=0, t=0):
    """Big-endian bytes of a w x h region of the plane."""
    y, x = np.mgrid[y0:y0 + h, x0:x0 + w].astype(np.int64)
    if kind == 1:  # G_FAKE
        v = TYPE_MIN[pt] + x
        box = x // 10
        special = (y < 10) & (box <= 4)
        vals = np.choose(np.clip(box, 0, 4), [0, plane_no, z, c, t])
        v = np.where(special, vals, v)
    else:
        xu, yu = x.astype(np.uint64), y.astype(np.uint64)
        k = (np.uint64(seed) << np.uint64(48)) ^ (np.uint64(plane_no) << np.uint64(40)) ^ \
            (yu << np.uint64(20)) ^ xu
        r = _splitmix(k)
        v = (256 + ((x >> 5) + (y >> 5)) % 16 * 48 + (r & np.uint64(0xFF)).astype(np.int64)
             + ((r >> np.uint64(8)) & np.uint64(0xFF)).astype(np.int64))
    return np.ascontiguousarray(_cast(pt, v)).tobytes()


def downsample(a):
    """One level of the resolution pyramid (include/pbx.h pbx_plane_build_pyramid), restated
    independently of csrc/kernels_io.hip: the 2x2 box mean, the last column / row repeated
    for odd sizes; integers (exact sum + 2) >> 2 (floor for signed), floats
    ((a + b) + (c + d)) * 0.25 in the array's precision.  `a`: 2-D array (any byte order)."""
    if a.shape[1] % 2:
        a = np.concatenate([a, a[:, -1:]], axis=1)
    if a.shape[0] % 2:
        a = np.concatenate([a, a[-1:, :]], axis=0)
    p, q, r, s = a[0::2, 0::2], a[0::2, 1::2], a[1::2, 0::2], a[1::2, 1::2]
    if a.dtype.kind == "f":
        return ((p + q) + (r + s)) * a.dtype.type(0.25)
    tot = p.astype(np.int64) + q.astype(np.int64) + r.astype(np.int64) + s.astype(np.int64)
    return ((tot + 2) >> 2).astype(a.dtype)
