"""The packed-f16 Paeth predictor of k_filter3 (kernels_io.hip paeth_pair_signs /
f3_paeth_word) restated in numpy half precision and checked against PNG's integer rule
(oracle/pbx_oracle.c, the reference's ImageIO PNG writer) for all 2^24 (left, up, up-left)
byte triples.

The kernel puts a byte x in a 16-bit lane under the byte 0x64: the f16 value 1024 + x, unit
steps in that exponent range, so every difference and sum the predictor forms is exact.  The
decisions are the sign bits of min(pb, pc) - pa and pc - pb (never -0: x - x = +0), turned into
byte masks by v_perm_b32's sign-replicating selectors, and two bitwise selects pick c over b,
then that over a.  This checks the arithmetic; the GPU tests check the kernel's bytes."""
import numpy as np


def _paeth_int(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def _paeth_f16(a, b, c):
    A = (1024 + a).astype(np.float16)
    B = (1024 + b).astype(np.float16)
    C = (1024 + c).astype(np.float16)
    d1 = B - C
    d2 = A - C
    d3 = d1 + d2
    pa, pb, pc = np.maximum(d1, -d1), np.maximum(d2, -d2), np.maximum(d3, -d3)
    na = np.signbit(np.minimum(pb, pc) - pa)   # pa > min(pb, pc)
    nb = np.signbit(pc - pb)                   # pb > pc
    t = np.where(nb, c, b)
    return np.where(na, t, a)


def test_paeth_f16_all_byte_triples():
    v = np.arange(256, dtype=np.int32)
    b, c = np.meshgrid(v, v, indexing="ij")
    b, c = b.ravel(), c.ravel()
    for a0 in range(0, 256, 32):  # 2^24 triples in eight slices of 2^21
        a = np.repeat(np.arange(a0, a0 + 32, dtype=np.int32), b.size)
        bb, cc = np.tile(b, 32), np.tile(c, 32)
        assert np.array_equal(_paeth_f16(a, bb, cc), _paeth_int(a, bb, cc))


def test_f16_differences_exact():
    # every value the predictor forms lies in [-510, 510]: integers there are exact in f16
    x = np.arange(-510, 511)
    assert np.array_equal(x.astype(np.float16).astype(np.int32), x)
