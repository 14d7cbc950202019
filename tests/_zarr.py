"""Zarr v2 chunk writers for the tests and the bench (test infrastructure only).

blosc_encode() writes c-blosc 1.x frames (format restated in oracle/zarr_oracle.c) with
LZ4 from the system liblz4 (the library c-blosc itself embeds) or zlib; zlib_encode() is a
Zarr "zlib" chunk.  The frame writer is checked against c-blosc 1.21 output
(tests/golden/zarr/, made by imagecodecs) in tests/test_zarr.py.
"""
import ctypes
import zlib

import numpy as np

_lz4 = None


def _liblz4():
    global _lz4
    if _lz4 is None:
        L = ctypes.CDLL("liblz4.so.1")
        L.LZ4_compressBound.argtypes = [ctypes.c_int]
        L.LZ4_compress_fast.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int]
        _lz4 = L
    return _lz4


def lz4_block(data: bytes, accel: int = 1) -> bytes:
    L = _liblz4()
    cap = L.LZ4_compressBound(len(data))
    out = ctypes.create_string_buffer(cap)
    n = L.LZ4_compress_fast(data, out, len(data), cap, accel)
    assert n > 0
    return out.raw[:n]


_zstd = None


def _libzstd():
    global _zstd
    if _zstd is None:
        L = ctypes.CDLL("libzstd.so.1")
        L.ZSTD_createCCtx.restype = ctypes.c_void_p
        L.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
        L.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.ZSTD_compressBound.restype = ctypes.c_size_t
        L.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
        L.ZSTD_compress2.restype = ctypes.c_size_t
        L.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                     ctypes.c_size_t]
        L.ZSTD_isError.argtypes = [ctypes.c_size_t]
        _zstd = L
    return _zstd


def zstd_frame(data: bytes, level: int = 5, checksum: bool = False) -> bytes:
    """One zstd frame from the system libzstd (ZSTD_c_compressionLevel = 100,
    ZSTD_c_checksumFlag = 201: the optional XXH64 content checksum)."""
    L = _libzstd()
    cc = L.ZSTD_createCCtx()
    try:
        L.ZSTD_CCtx_setParameter(cc, 100, level)
        L.ZSTD_CCtx_setParameter(cc, 201, 1 if checksum else 0)
        cap = L.ZSTD_compressBound(len(data))
        out = ctypes.create_string_buffer(cap)
        n = L.ZSTD_compress2(cc, out, cap, data, len(data))
        assert not L.ZSTD_isError(n)
        return out.raw[:n]
    finally:
        L.ZSTD_freeCCtx(cc)


def blosc_blocksize(nbytes: int, typesize: int, clevel: int, codec: str) -> int:
    """c-blosc 1.21 compute_blocksize() for the automatic block size."""
    L1 = 32 * 1024
    bs = nbytes
    if nbytes >= L1:
        bs = L1
        if codec in ("lz4hc", "zlib", "zstd"):
            bs *= 2
        bs = {0: bs // 4, 1: bs // 2, 2: bs, 3: bs * 2, 4: bs * 4, 5: bs * 4, 6: bs * 8, 7: bs * 8,
              8: bs * 8, 9: bs * 8 * (2 if codec in ("lz4hc", "zlib", "zstd") else 1)}[clevel]
    if clevel > 0 and codec != "zstd" and typesize <= 16 and bs // typesize >= 128:
        bs = min(bs, 1 << 18) * typesize
        bs = max(bs, 1 << 16)
        bs = min(bs, 1 << 18)
    if bs > nbytes:
        bs = nbytes
    if bs > typesize:
        bs = bs // typesize * typesize
    return bs


def shuffle_block(block: bytes, ts: int) -> bytes:
    n = len(block) // ts
    a = np.frombuffer(block[:n * ts], dtype=np.uint8).reshape(n, ts)
    return a.T.tobytes() + block[n * ts:]


def blosc_encode(raw: bytes, typesize: int, clevel: int = 5, shuffle: bool = True,
                 codec: str = "lz4", blocksize: int = 0, split: bool = True,
                 zstd_checksum: bool = False) -> bytes:
    nbytes = len(raw)
    ts = max(1, typesize)
    bs = blocksize or blosc_blocksize(nbytes, ts, clevel, codec)
    bs = max(1, min(bs, nbytes))
    nblocks = -(-nbytes // bs)
    leftover = nbytes % bs
    compcode = {"lz4": 1, "lz4hc": 1, "zlib": 3, "zstd": 4}[codec]
    flags = (0x1 if shuffle else 0) | (compcode << 5) | (0 if split else 0x10)
    body = bytearray()
    starts = []
    hdr = 16 + 4 * nblocks
    for b in range(nblocks):
        is_left = leftover and b == nblocks - 1
        bsize = leftover if is_left else bs
        block = raw[b * bs:b * bs + bsize]
        if shuffle and ts > 1:
            block = shuffle_block(block, ts)
        nsp = ts if (split and ts <= 16 and bsize // ts >= 128 and not is_left) else 1
        neb = bsize // nsp
        starts.append(hdr + len(body))
        for s in range(nsp):
            part = block[s * neb:(s + 1) * neb]
            if codec == "zstd":  # (zstd_checksum: frames carrying XXH64 content checksums)
                c = zstd_frame(part, clevel, zstd_checksum)
            else:
                c = lz4_block(part, max(1, 10 - clevel)) if codec != "zlib" else zlib.compress(part, clevel)
            if len(c) >= neb:
                c = part
            body += len(c).to_bytes(4, "little") + c
    cbytes = hdr + len(body)
    if cbytes >= nbytes + 16:  # memcpyed frame
        flags |= 0x2
        return bytes([2, 1, flags, ts]) + nbytes.to_bytes(4, "little") + bs.to_bytes(4, "little") + \
            (nbytes + 16).to_bytes(4, "little") + raw
    out = bytes([2, 1, flags, ts]) + nbytes.to_bytes(4, "little") + bs.to_bytes(4, "little") + \
        cbytes.to_bytes(4, "little") + b"".join(x.to_bytes(4, "little") for x in starts) + bytes(body)
    return out


def zlib_encode(raw: bytes, level: int = 1) -> bytes:
    return zlib.compress(raw, level)


def chunk_grid(plane: np.ndarray, chunk_y: int, chunk_x: int):
    """C-order list of full-size (edge-padded with zeros) chunk arrays of a 2-D plane."""
    sy, sx = plane.shape
    out = []
    for j in range(-(-sy // chunk_y)):
        for i in range(-(-sx // chunk_x)):
            c = np.zeros((chunk_y, chunk_x), dtype=plane.dtype)
            blk = plane[j * chunk_y:(j + 1) * chunk_y, i * chunk_x:(i + 1) * chunk_x]
            c[:blk.shape[0], :blk.shape[1]] = blk
            out.append(c)
    return out


# The real c-blosc 1.21.0 (the image's /opt/conda libblosc, the library imagecodecs and
# numcodecs wrap), used to ENCODE test chunks with every codec and shuffle mode (blosclz,
# lz4, lz4hc, zlib, zstd; no / byte / bit shuffle) and, in CPU tests, to decode them as a
# second reference next to oracle/zarr_oracle.c.  Test infrastructure only.
CBLOSC_PATH = "/opt/conda/lib/libblosc.so.1"
_cb = None


def cblosc():
    """ctypes handle of c-blosc 1.21 or None when the image lacks it."""
    global _cb
    if _cb is None:
        import os
        if not os.path.exists(CBLOSC_PATH):
            _cb = False
            return None
        L = ctypes.CDLL(CBLOSC_PATH)
        L.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
        L.blosc_decompress_ctx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _cb = L
    return _cb or None


def cblosc_encode(raw: bytes, typesize: int, cname: str = "lz4", clevel: int = 5, shuffle: int = 1,
                  blocksize: int = 0) -> bytes:
    """blosc_compress_ctx (shuffle 0 none, 1 byte, 2 bit)."""
    L = cblosc()
    out = ctypes.create_string_buffer(len(raw) + 64)
    n = L.blosc_compress_ctx(clevel, shuffle, typesize, len(raw), raw, out, len(out), cname.encode(),
                             blocksize, 1)
    assert n > 0, (cname, n)
    return out.raw[:n]


def cblosc_decode(enc: bytes, nbytes: int) -> bytes:
    L = cblosc()
    out = ctypes.create_string_buffer(max(nbytes, 1))
    n = L.blosc_decompress_ctx(enc, out, nbytes, 1)
    assert n == nbytes, n
    return out.raw[:nbytes]


def encode_chunks(plane: np.ndarray, chunk_y: int, chunk_x: int, compressor, **kw):
    """Chunk files of a plane for the .zarray compressor id (None, "blosc", "zlib");
    kw: blosc_encode options (codec, clevel, shuffle, blocksize, split) or zlib level; with
    cname=... the chunks come from the real c-blosc (cblosc_encode options)."""
    out = []
    for c in chunk_grid(plane, chunk_y, chunk_x):
        raw = c.tobytes()
        if compressor == "blosc" and "cname" in kw:
            out.append(cblosc_encode(raw, c.dtype.itemsize, **kw))
        elif compressor == "blosc":
            out.append(blosc_encode(raw, c.dtype.itemsize, **kw))
        elif compressor == "zlib":
            out.append(zlib_encode(raw, kw.get("level", 1)))
        else:
            out.append(raw)
    return out


def noise_plane(h: int, w: int, dtype=">u2", seed: int = 0) -> np.ndarray:
    """G_NOISE-like 12-bit image: blocky background + 9-bit noise."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    v = 256 + ((x >> 5) + (y >> 5)) % 16 * 48 + rng.integers(0, 512, size=(h, w))
    return v.astype(dtype)
