"""ctypes binding of lib/libpbx_emu.so: TEST-ONLY CPU emulation of the deflate workgroup."""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "omero-ms-pixel-buffer_amd", "lib", "libpbx_emu.so")


class SegOut(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in
                "nbytes crc crc_op adler_s1 adler_s2 len btype bits".split()]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB_PATH)
        L.pbxemu_deflate.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(SegOut)]
        L.pbxemu_nsegs.restype = ctypes.c_uint32
        L.pbxemu_nsegs.argtypes = [ctypes.c_uint64]
        L.pbxemu_nblocks.restype = ctypes.c_uint32
        L.pbxemu_nblocks.argtypes = [ctypes.c_uint64]
        L.pbxemu_huffman.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.pbxemu_lz77.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_void_p]
        L.pbxemu_hist_words.restype = ctypes.c_uint32
        L.pbxemu_mrec_words.restype = ctypes.c_uint32
        L.pbxemu_crc_combine.restype = ctypes.c_uint32
        L.pbxemu_crc_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.pbxemu_crc_fast_mismatches.restype = ctypes.c_uint64
        L.pbxemu_rle_closed_mismatches.restype = ctypes.c_uint32
        L.pbxemu_crc_fast_mismatches.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        _lib = L
    return _lib


def deflate(data: bytes, rowlen: int):
    """zlib stream exactly as the GPU pipeline produces it for one tile stream, and the
    per-block results (SegOut per deflate block)."""
    data = bytes(data)
    n = lib().pbxemu_nblocks(len(data))
    segs = (SegOut * n)()
    out = ctypes.create_string_buffer(len(data) + 1024 + 16 * n)
    ol = ctypes.c_uint64()
    r = lib().pbxemu_deflate(data, len(data), rowlen, out, len(out), ctypes.byref(ol), segs)
    assert r == 0, r
    return out.raw[: ol.value], list(segs)


def crc_combine(c1, c2, len2):
    return lib().pbxemu_crc_combine(c1, c2, len2)


def crc_fast_mismatches(n, seed):
    return lib().pbxemu_crc_fast_mismatches(n, seed)


def rle_closed_mismatches():
    return lib().pbxemu_rle_closed_mismatches()


def huffman(hist, sl, last):
    """Huffman stage alone: (codes[480], info[4]) as uint32 numpy arrays."""
    import numpy as np
    h = np.ascontiguousarray(hist, dtype=np.uint32)
    assert h.shape == (320,)
    codes = np.zeros(480, np.uint32)
    info = np.zeros(4, np.uint32)
    r = lib().pbxemu_huffman(h.ctypes.data, sl, last, codes.ctypes.data, info.ctypes.data)
    assert r == 0
    return codes, info


def lz77(data: bytes, rowlen: int):
    """LZ77 stage alone: (hist[nseg, 320], mrec[nseg, MREC_WORDS]) as k_lz77 writes them."""
    import numpy as np
    data = bytes(data)
    L = lib()
    n = L.pbxemu_nsegs(len(data))
    hw, mw = L.pbxemu_hist_words(), L.pbxemu_mrec_words()
    h = np.zeros(n * hw, np.uint32)
    m = np.zeros(n * mw, np.uint32)
    r = L.pbxemu_lz77(data, len(data), rowlen, h.ctypes.data, m.ctypes.data)
    assert r == 0, r
    return h.reshape(n, hw), m.reshape(n, mw)
