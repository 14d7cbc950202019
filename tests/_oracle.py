"""ctypes binding of the CPU oracle (oracle/pbx_oracle.c) — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "libpbx_oracle.so")

INT8, UINT8, INT16, UINT16, INT32, UINT32, FLOAT, DOUBLE = range(8)
TYPE_NAMES = ["int8", "uint8", "int16", "uint16", "int32", "uint32", "float", "double"]
BPP = [1, 1, 2, 2, 4, 4, 4, 8]
NP_BE = [">i1", ">u1", ">i2", ">u2", ">i4", ">u4", ">f4", ">f8"]
FMT_RAW, FMT_PNG, FMT_TIF, FMT_UNKNOWN = range(4)
GEN_FAKE, GEN_NOISE = 1, 2

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        szp = ctypes.POINTER(ctypes.c_size_t)
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.pbxo_gen_region.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                      ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                                      u8p]
        L.pbxo_gen_sample.restype = ctypes.c_uint64
        L.pbxo_gen_sample.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                      ctypes.c_int64]
        L.pbxo_extract_be.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, u8p]
        L.pbxo_png_filter_stream.restype = ctypes.c_size_t
        L.pbxo_png_filter_stream.argtypes = [u8p, ctypes.c_int, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int, u8p]
        L.pbxo_adaptive_tile_none.argtypes = [u8p, ctypes.c_int, ctypes.c_int32, ctypes.c_int32]
        L.pbxo_png_encode.argtypes = [u8p, ctypes.c_int, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int, u8p, ctypes.c_size_t, szp]
        L.pbxo_tiff_encode.argtypes = [u8p, ctypes.c_int, ctypes.c_int32, ctypes.c_int32, u8p,
                                       ctypes.c_size_t, szp]
        L.pbxo_png_max_size.restype = ctypes.c_size_t
        L.pbxo_png_max_size.argtypes = [ctypes.c_int, ctypes.c_int32, ctypes.c_int32]
        L.pbxo_tiff_size.restype = ctypes.c_size_t
        L.pbxo_tiff_size.argtypes = [ctypes.c_int, ctypes.c_int32, ctypes.c_int32]
        L.pbxo_get_tile.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_int, u8p,
                                    ctypes.c_size_t, szp, i32p, i32p]
        L.pbxo_png_decode.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, i32p, i32p,
                                      i32p, i32p]
        L.pbxo_png_inflate_idat.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, szp]
        L.pbxo_tiff_decode.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, i32p, i32p,
                                       i32p, i32p, i32p, i32p]
        L.pbxo_zlib_inflate.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, szp]
        L.pbxo_tiff_tiled_write.argtypes = [u8p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, u8p,
                                            ctypes.c_size_t, szp]
        L.pbxo_crc32.restype = ctypes.c_uint32
        L.pbxo_crc32.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.pbxo_adler32.restype = ctypes.c_uint32
        L.pbxo_adler32.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.pbxo_tile_filename.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                                         ctypes.c_char_p, ctypes.c_size_t]
        L.pbxo_content_type.restype = ctypes.c_char_p
        L.pbxo_content_type.argtypes = [ctypes.c_char_p]
        L.pbxo_bench.restype = ctypes.c_double
        L.pbxo_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int32,
                                 ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                                 ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.pbxo_bench_at.restype = ctypes.c_double
        L.pbxo_bench_at.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def gen_region(kind, pt, x0, y0, w, h, seed=0, plane_no=0, z=0, c=0, t=0, big_endian=True):
    out = np.zeros(w * h * BPP[pt], np.uint8)
    lib().pbxo_gen_region(kind, seed, plane_no, z, c, t, pt, x0, y0, w, h, int(big_endian), _p(out))
    return out


def extract_be(plane, plane_be, pt, pitch, x, y, w, h):
    out = np.zeros(w * h * BPP[pt], np.uint8)
    plane = np.ascontiguousarray(plane).view(np.uint8).reshape(-1)
    lib().pbxo_extract_be(_p(plane), int(plane_be), pt, pitch, x, y, w, h, _p(out))
    return out


def png_filter_stream(tile_be, pt, w, h, filt=0):
    out = np.zeros(h * (1 + w * BPP[pt]), np.uint8)
    lib().pbxo_png_filter_stream(_p(tile_be), pt, w, h, filt, _p(out))
    return out


def adaptive_tile_none(tile_be, pt, w, h):
    """The adaptive option's tile mode: True when every row of the tile takes filter None."""
    return bool(lib().pbxo_adaptive_tile_none(_p(tile_be), pt, w, h))


def png_encode(tile_be, pt, w, h, level=6):
    cap = lib().pbxo_png_max_size(pt, w, h)
    out = np.zeros(cap, np.uint8)
    n = ctypes.c_size_t()
    st = lib().pbxo_png_encode(_p(tile_be), pt, w, h, level, _p(out), cap, ctypes.byref(n))
    return st, bytes(out[: n.value]) if st == 0 else None


def tiff_encode(tile_be, pt, w, h):
    cap = lib().pbxo_tiff_size(pt, w, h)
    out = np.zeros(cap, np.uint8)
    n = ctypes.c_size_t()
    st = lib().pbxo_tiff_encode(_p(tile_be), pt, w, h, _p(out), cap, ctypes.byref(n))
    return st, bytes(out[: n.value]) if st == 0 else None


def get_tile(plane, plane_be, pt, sx, sy, x, y, w, h, fmt):
    ww = w if w else sx
    hh = h if h else sy
    cap = max(1, ww * hh * BPP[pt]) * 2 + 4096 if ww > 0 and hh > 0 and ww * hh < (1 << 31) else 16
    if fmt == FMT_PNG and ww > 0 and hh > 0 and ww * hh < (1 << 31):
        cap = max(cap, lib().pbxo_png_max_size(pt, ww, hh))
    out = np.zeros(cap, np.uint8)
    n = ctypes.c_size_t()
    ow, oh = ctypes.c_int32(), ctypes.c_int32()
    plane = np.ascontiguousarray(plane).view(np.uint8).reshape(-1)
    st = lib().pbxo_get_tile(_p(plane), int(plane_be), pt, sx, sy, x, y, w, h, fmt, _p(out), cap,
                             ctypes.byref(n), ctypes.byref(ow), ctypes.byref(oh))
    return st, (bytes(out[: n.value]) if st == 0 else None), ow.value, oh.value


def png_decode(buf):
    a = np.frombuffer(buf, np.uint8).copy()
    w, h, d, ct = (ctypes.c_int32() for _ in range(4))
    # first pass for size
    cap = 1 << 20
    while True:
        out = np.zeros(cap, np.uint8)
        r = lib().pbxo_png_decode(_p(a), len(a), _p(out), cap, ctypes.byref(w), ctypes.byref(h),
                                  ctypes.byref(d), ctypes.byref(ct))
        if r == -8:
            cap = w.value * h.value * (d.value // 8) + 16
            continue
        break
    if r != 0:
        return r, None, None
    n = w.value * h.value * (d.value // 8)
    return 0, bytes(out[:n]), dict(w=w.value, h=h.value, depth=d.value, color_type=ct.value)


def png_inflate_idat(buf, cap):
    a = np.frombuffer(buf, np.uint8).copy()
    out = np.zeros(cap + 1, np.uint8)
    n = ctypes.c_size_t()
    r = lib().pbxo_png_inflate_idat(_p(a), len(a), _p(out), cap + 1, ctypes.byref(n))
    return r, bytes(out[: n.value]) if r == 0 else None


def tiff_decode(buf, cap):
    a = np.frombuffer(buf, np.uint8).copy()
    out = np.zeros(max(cap, 1), np.uint8)
    v = [ctypes.c_int32() for _ in range(6)]
    r = lib().pbxo_tiff_decode(_p(a), len(a), _p(out), cap, *[ctypes.byref(x) for x in v])
    meta = dict(zip(["w", "h", "bits", "sample_format", "compression", "big_endian"],
                    [x.value for x in v]))
    if r != 0:
        return r, None, meta
    n = meta["w"] * meta["h"] * meta["bits"] // 8
    return 0, bytes(out[:n]), meta


def tiff_tiled_write(tile_be, w, h, bpp, sf, t, comp):
    """Tiled TIFF of the big-endian tile bytes (the pipeline's tiled-TIFF layout)."""
    a = np.ascontiguousarray(np.frombuffer(bytes(tile_be), np.uint8))
    ntx, nty = -(-w // t), -(-h // t)
    cap = 256 + 8 * ntx * nty + 2 * ntx * nty * (t * t * bpp + 64)
    out = np.zeros(cap, np.uint8)
    n = ctypes.c_size_t()
    r = lib().pbxo_tiff_tiled_write(_p(a), w, h, bpp, sf, t, comp, _p(out), cap, ctypes.byref(n))
    if r != 0:
        raise ValueError(f"pbxo_tiff_tiled_write: {r}")
    return bytes(out[: n.value])


def zlib_inflate(buf, cap):
    a = np.frombuffer(buf, np.uint8).copy()
    out = np.zeros(cap + 1, np.uint8)
    n = ctypes.c_size_t()
    r = lib().pbxo_zlib_inflate(_p(a), len(a), _p(out), cap + 1, ctypes.byref(n))
    return r, bytes(out[: n.value]) if r == 0 else None


def tile_filename(image_id, z, c, t, x, y, w, h, fmt):
    buf = ctypes.create_string_buffer(256)
    lib().pbxo_tile_filename(image_id, z, c, t, x, y, w, h,
                             fmt.encode() if fmt is not None else None, buf, 256)
    return buf.value.decode()


def content_type(fmt):
    return lib().pbxo_content_type(fmt.encode() if fmt is not None else None).decode()


def bench(kind, pt, fmt, pw, ph, w, h, tiles, threads):
    nb = ctypes.c_uint64()
    sec = lib().pbxo_bench(kind, pt, fmt, pw, ph, w, h, tiles, threads, ctypes.byref(nb))
    return sec, nb.value


def bench_at(kind, pt, fmt, pw, ph, x, y, w, h, reps, threads):
    nb = ctypes.c_uint64()
    sec = lib().pbxo_bench_at(kind, pt, fmt, pw, ph, x, y, w, h, reps, threads, ctypes.byref(nb))
    return sec, nb.value


def check_png_grid_pixels(bodies, pt, tile_w, tile_h, grid_x, y_row0, kind=2, seed=0, threads=8):
    """Pixel check of EVERY tile of a grid of filter-None PNG responses (PNG of 8/16-bit
    unsigned samples), tile i at (tile_w * (i % grid_x), y_row0 + tile_h * (i // grid_x)):
    each IDAT is inflated by zlib and its scanlines, filter bytes stripped, must equal the
    oracle generator's big-endian tile.  One oracle band per grid row (threads in parallel).
    Returns the indices of the tiles that differ."""
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    bpp = BPP[pt]
    rows = (len(bodies) + grid_x - 1) // grid_x

    def row(r):
        band = gen_region(kind, pt, 0, y_row0 + r * tile_h, tile_w * grid_x, tile_h, seed=seed)
        band = band.reshape(tile_h, tile_w * grid_x * bpp)
        bad = []
        for i in range(r * grid_x, min(len(bodies), (r + 1) * grid_x)):
            b = bodies[i]
            x = i % grid_x
            try:
                n = int.from_bytes(b[91:95], "big")
                scan = np.frombuffer(zlib.decompress(b[99:99 + n]), np.uint8)
                scan = scan.reshape(tile_h, 1 + tile_w * bpp)
                ok = not scan[:, 0].any() and np.array_equal(
                    scan[:, 1:], band[:, x * tile_w * bpp:(x + 1) * tile_w * bpp])
            except Exception:
                ok = False
            if not ok:
                bad.append(i)
        return bad

    with ThreadPoolExecutor(threads) as ex:
        return [i for part in ex.map(row, range(rows)) for i in part]
