"""Regions at every source alignment: the reference serves any x, y
(TileCtx.java:73-85; getTileDirect, TileRequestHandler.java:98-109), so most requests start at
a byte offset x * bpp that is not a multiple of 16.  k_extract (raw, TIFF) and the staged PNG
row kernel (k_filter) read such rows as aligned 16-byte words realigned in registers
(gload16u); these tests sweep x mod 16 x the 8 pixel types x odd widths (row lengths below,
around and far above 16 bytes, rows of one workgroup each) x both plane byte orders, and
compare every response with the oracle's getTile restatement (oracle/pbx_oracle.c, the
checker only): raw and uncompressed TIFF byte-identical, PNG inflating to the oracle's
scanlines for every filter mode.
"""
import itertools

import numpy as np
import pytest

import pbx

pytestmark = pytest.mark.gpu

_ids = itertools.count(810000)
SX, SY = 2112, 80


def _planes(svc, oracle, pts):
    out = {}
    for pt in pts:
        for be in (True, False):
            iid = next(_ids)
            plane_be = oracle.gen_region(2, pt, 0, 0, SX, SY, seed=pt, big_endian=True)
            data = plane_be if be else oracle.gen_region(2, pt, 0, 0, SX, SY, seed=pt, big_endian=False)
            svc.register_plane(iid, 0, 0, 0, pt, SX, SY, data=data, big_endian=be)
            out[(pt, be)] = (iid, plane_be)
    return out


def _check(oracle, planes, meta, res, png_filter=0):
    n = 0
    for (pt, be, x, y, w, h, fmt), (st, body) in zip(meta, res):
        fcode = {None: oracle.FMT_RAW, "png": oracle.FMT_PNG, "tif": oracle.FMT_TIF}[fmt]
        plane_be = planes[(pt, be)][1]
        ost, obody, ow, oh = oracle.get_tile(plane_be, True, pt, SX, SY, x, y, w, h, fcode)
        assert st == (pbx.OK if ost == 0 else ost), (pt, be, x, y, w, h, fmt, st, ost)
        if st != pbx.OK:
            continue
        n += 1
        if fmt != "png":
            assert body == obody, (pt, be, x, y, w, h, fmt)
            continue
        tile = oracle.extract_be(plane_be, True, pt, SX * oracle.BPP[pt], x, y, w, h)
        stream = oracle.png_filter_stream(tile, pt, w, h, png_filter).tobytes()
        r, idat = oracle.png_inflate_idat(body, len(stream))
        assert r == 0 and idat == stream, (pt, be, x, y, w, h, png_filter)
    return n


def test_unaligned_sweep_raw_tif_png(oracle):
    """x = 0..15 (every x * bpp mod 16) x 8 pixel types x widths {3, 9, 17, 100, 513, 2053}
    (rows of 3 B to 16 KiB: several rows per k_extract workgroup, one row per workgroup) x
    heights {1, 7, 70} x raw / tif / png x both byte orders, all in one batch."""
    with pbx.PixelsService() as svc:
        planes = _planes(svc, oracle, range(8))
        ctxs, meta = [], []
        for pt, be, x, w in itertools.product(range(8), (True, False), range(16), (3, 9, 17, 100, 513, 2053)):
            for k, fmt in enumerate((None, "tif", "png")):
                h = (1, 7, 70)[(x + k + w) % 3]
                y = (x * 5 + k) % (SY - h + 1)
                ctxs.append(pbx.TileCtx(planes[(pt, be)][0], 0, 0, 0, x, y, w, h, format=fmt))
                meta.append((pt, be, x, y, w, h, fmt))
        res = svc.get_tiles(ctxs)
        n = _check(oracle, planes, meta, res)
    assert n > 0.8 * len(ctxs)  # PNG of 32/64-bit types: the reference's 404


@pytest.mark.parametrize("png_filter", [1, 2, 3, 4, 5], ids=["sub", "up", "avg", "paeth", "adaptive"])
def test_unaligned_png_filters(oracle, png_filter):
    """The staged PNG rows (k_filter) at every source alignment under each PNG filter: 8- and
    16-bit types, x = 0..15, widths from 5 to 1031 samples."""
    with pbx.PixelsService(png_filter=png_filter) as svc:
        planes = _planes(svc, oracle, (pbx.INT8, pbx.UINT8, pbx.INT16, pbx.UINT16))
        ctxs, meta = [], []
        for pt, be, x, w in itertools.product((pbx.INT8, pbx.UINT8, pbx.INT16, pbx.UINT16), (True, False),
                                               range(16), (5, 33, 250, 1031)):
            h = 3 + (x * 7 + w) % 40
            y = (x * 3 + w) % (SY - h + 1)
            ctxs.append(pbx.TileCtx(planes[(pt, be)][0], 0, 0, 0, x, y, w, h, format="png"))
            meta.append((pt, be, x, y, w, h, "png"))
        res = svc.get_tiles(ctxs)
        assert _check(oracle, planes, meta, res, png_filter) == len(ctxs)


def test_unaligned_full_size_tiles(oracle):
    """configs[4]-sized regions at odd x: 1000..2048-px uint8 / int32 / float32 tiles of a
    4096^2 plane, x * bpp mod 16 != 0, raw / tif / png, every response against the oracle."""
    side = 4096
    rng = np.random.default_rng(66)
    with pbx.PixelsService() as svc:
        host, ids = {}, {}
        for pt in (pbx.UINT8, pbx.INT32, pbx.FLOAT):
            ids[pt] = next(_ids)
            svc.register_plane(ids[pt], 0, 0, 0, pt, side, side, generator="noise", seed=0)
            host[pt] = oracle.gen_region(2, pt, 0, 0, side, side)
        ctxs, meta = [], []
        for k in range(48):
            pt = (pbx.UINT8, pbx.INT32, pbx.FLOAT)[k % 3]
            w, h = int(rng.integers(1000, 2049)), int(rng.integers(256, 1025))
            x = int(rng.integers(0, side - w)) | 1
            y = int(rng.integers(0, side - h + 1))
            fmt = (None, "tif", "png")[(k // 3) % 3]
            ctxs.append(pbx.TileCtx(ids[pt], 0, 0, 0, x, y, w, h, format=fmt))
            meta.append((pt, x, y, w, h, fmt))
        res = svc.get_tiles(ctxs)
    for (pt, x, y, w, h, fmt), (st, body) in zip(meta, res):
        fcode = {None: oracle.FMT_RAW, "png": oracle.FMT_PNG, "tif": oracle.FMT_TIF}[fmt]
        ost, obody, _, _ = oracle.get_tile(host[pt], True, pt, side, side, x, y, w, h, fcode)
        assert st == (pbx.OK if ost == 0 else ost), (pt, x, y, w, h, fmt)
        if st != pbx.OK:
            continue
        if fmt == "png":
            tile = oracle.extract_be(host[pt], True, pt, side * oracle.BPP[pt], x, y, w, h)
            stream = oracle.png_filter_stream(tile, pt, w, h, 0).tobytes()
            r, idat = oracle.png_inflate_idat(body, len(stream))
            assert r == 0 and idat == stream, (pt, x, y, w, h)
        else:
            assert body == obody, (pt, x, y, w, h, fmt)


def test_pipelined_mixed_batches_split_extract(oracle):
    """Pipelined device-resident batches (pbx_batch_launch: the bench's form) that hold raw /
    TIFF tiles next to PNG tiles run their k_extract on the context's extract stream beside
    the deflate chain (runtime.cpp pbx_ctx::xstream); four such batches in flight at once,
    every response against the oracle."""
    side = 4096
    rng = np.random.default_rng(67)
    with pbx.PixelsService() as svc:
        host, ids = {}, {}
        for pt in (pbx.UINT8, pbx.INT32, pbx.FLOAT):
            ids[pt] = next(_ids)
            svc.register_plane(ids[pt], 0, 0, 0, pt, side, side, generator="noise", seed=0)
            host[pt] = oracle.gen_region(2, pt, 0, 0, side, side)
        batches = []
        for _ in range(4):
            ctxs, meta = [], []
            for k in range(96):
                pt = (pbx.UINT8, pbx.INT32, pbx.FLOAT)[int(rng.integers(3))]
                w, h = int(rng.integers(1, 5)) * 256, int(rng.integers(1, 5)) * 256
                x, y = int(rng.integers(0, side - w + 1)), int(rng.integers(0, side - h + 1))
                fmt = (None, "tif", "png")[int(rng.integers(3))]
                ctxs.append(pbx.TileCtx(ids[pt], 0, 0, 0, x, y, w, h, format=fmt))
                meta.append((pt, x, y, w, h, fmt))
            batches.append((pbx.Batch(svc, ctxs), meta))
        for b, _ in batches:  # all four launched before any is waited for
            b.launch()
        results = []
        for b, meta in batches:
            b.sync()
            results.append((b.fetch(), meta))
            b.close()
    n = 0
    for res, meta in results:
        for (pt, x, y, w, h, fmt), (st, body) in zip(meta, res):
            fcode = {None: oracle.FMT_RAW, "png": oracle.FMT_PNG, "tif": oracle.FMT_TIF}[fmt]
            ost, obody, _, _ = oracle.get_tile(host[pt], True, pt, side, side, x, y, w, h, fcode)
            assert st == (pbx.OK if ost == 0 else ost), (pt, x, y, w, h, fmt)
            if st != pbx.OK:
                continue
            n += 1
            if fmt == "png":
                tile = oracle.extract_be(host[pt], True, pt, side * oracle.BPP[pt], x, y, w, h)
                stream = oracle.png_filter_stream(tile, pt, w, h, 0).tobytes()
                r, idat = oracle.png_inflate_idat(body, len(stream))
                assert r == 0 and idat == stream, (pt, x, y, w, h)
            else:
                assert body == obody, (pt, x, y, w, h, fmt)
    assert n > 250
