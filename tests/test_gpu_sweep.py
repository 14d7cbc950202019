"""GPU parity at full size (> 4 GiB plane offsets) and a seeded random sweep.

* configs[2]'s 65536^2 uint16 plane (8 GiB): tiles whose source rows lie above 4 GiB
  (y >= 32768) as PNG, raw and TIFF, bit-exact against the oracle's generator;
* configs[3]'s 100000^2 uint16 plane (20 GB): the last tile-row band (160-px edge tiles) and
  the corner tile as TIFF, byte-identical to the oracle's TIFF;
* a seeded sweep over pixel type x format x plane byte order x odd x/y/w/h x PNG filter
  mode, every response compared with the oracle's getTile restatement
  (oracle/pbx_oracle.c pbxo_get_tile): same status; raw and uncompressed TIFF byte-identical;
  PNG decoding to the same pixels and inflating to the oracle's filtered scanlines.

Reference: TileRequestHandler.java:80-139 (getTile), :98-128 (getTileDirect + writeImage).
"""
import itertools
import zlib

import numpy as np
import pytest

import pbx

pytestmark = pytest.mark.gpu

_ids = itertools.count(700000)


def _flip(tile, pt):
    a = bytearray(tile)
    if pt in (pbx.INT8, pbx.INT16):
        a[0::pbx.BYTES_PER_PIXEL[pt]] = bytes(b ^ 0x80 for b in a[0::pbx.BYTES_PER_PIXEL[pt]])
    return bytes(a)


def test_plane_above_4gib(service, oracle):
    """65536^2 uint16 (8 GiB, configs[2]): every byte offset of these tiles is >= 4 GiB."""
    iid = next(_ids)
    side = 65536
    pid = service.register_plane(iid, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0)
    try:
        regions = [(65024, 65024, 512, 512, "png"), (0, 32768, 1024, 1024, "png"),
                   (12345, 50001, 513, 257, "png"), (65535, 65535, 1, 1, "png"),
                   (40000, 40000, 512, 512, None), (7, 60001, 333, 97, None),
                   (65536 - 160, 32768, 160, 512, "tif"), (31, 65000, 1000, 536, "tif")]
        ctxs = [pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format=f) for x, y, w, h, f in regions]
        # and a 64-tile grid row of 1024^2 PNG tiles in the top half of the plane
        grid = [pbx.TileCtx(iid, 0, 0, 0, 1024 * i, 63 * 1024, 1024, 1024, format="png")
                for i in range(64)]
        res = service.get_tiles(ctxs + grid)
        for (x, y, w, h, f), (st, body) in zip(regions, res):
            assert st == pbx.OK, (x, y, w, h, f)
            tile = oracle.gen_region(2, pbx.UINT16, x, y, w, h).tobytes()
            if f is None:
                assert body == tile, (x, y)
            elif f == "tif":
                assert body == oracle.tiff_encode(np.frombuffer(tile, np.uint8).copy(),
                                                  pbx.UINT16, w, h)[1], (x, y)
            else:
                r, px, meta = oracle.png_decode(body)
                assert r == 0 and px == tile and (meta["w"], meta["h"]) == (w, h), (x, y)
        # every tile of the grid row pixel-checked against the oracle
        assert all(st == pbx.OK for st, _ in res[len(regions):])
        bodies = [b for _, b in res[len(regions):]]
        assert oracle.check_png_grid_pixels(bodies, pbx.UINT16, 1024, 1024, 64, 63 * 1024) == []
        r, px, _ = oracle.png_decode(bodies[63])
        assert r == 0 and px == oracle.gen_region(2, pbx.UINT16, 1024 * 63, 63 * 1024, 1024, 1024).tobytes()
    finally:
        service.release_plane(pid)


def test_wholeslide_100k_last_band(service, oracle):
    """configs[3]: a 100000^2 uint16 channel (20 GB).  The last tile-row band (tiles 512 x 160)
    and the 160 x 160 corner tile are byte-identical to the oracle's TIFFs."""
    iid = next(_ids)
    side, n = 100000, (100000 + 511) // 512
    pid = service.register_plane(iid, 0, 4, 0, pbx.UINT16, side, side, generator="noise",
                                 seed=0, plane_no=4)
    try:
        ty = n - 1
        ctxs = [pbx.TileCtx(iid, 0, 4, 0, 512 * tx, 512 * ty, min(512, side - 512 * tx),
                            side - 512 * ty, format="tif") for tx in range(n)]
        ctxs.append(pbx.TileCtx(iid, 0, 4, 0, 512 * 97, 512 * 101, 512, 512, format="tif"))
        res = service.get_tiles(ctxs)
        for c, (st, body) in zip(ctxs, res):
            assert st == pbx.OK
            tile = oracle.gen_region(2, pbx.UINT16, c.x, c.y, c.w, c.h, plane_no=4, c=4)
            assert body == oracle.tiff_encode(tile, pbx.UINT16, c.w, c.h)[1], (c.x, c.y)
        assert (ctxs[-2].w, ctxs[-2].h) == (160, 160)
    finally:
        service.release_plane(pid)


FILTERS = [pbx.FILTER_NONE, pbx.FILTER_SUB, pbx.FILTER_UP, pbx.FILTER_AVG, pbx.FILTER_PAETH,
           pbx.FILTER_ADAPTIVE]


@pytest.mark.parametrize("png_filter", FILTERS, ids=["none", "sub", "up", "avg", "paeth", "adaptive"])
def test_random_sweep(oracle, png_filter):
    """Seeded sweep: 8 pixel types x 2 byte orders x {raw, png, tif, bad format} x odd regions
    (some outside the plane, w/h = 0 defaults) for one PNG filter mode, all requests in one
    batch, every response against the oracle's getTile."""
    rng = np.random.default_rng(1000 + png_filter)
    sx, sy = 613, 211
    with pbx.PixelsService(png_filter=png_filter, tiff_deflate=png_filter == pbx.FILTER_ADAPTIVE) as svc:
        planes = {}
        for pt in range(8):
            for be in (True, False):
                iid = next(_ids)
                kind = 1 + int(rng.integers(2))
                plane_be = oracle.gen_region(kind, pt, 0, 0, sx, sy, seed=pt, big_endian=True)
                data = plane_be if be else oracle.gen_region(kind, pt, 0, 0, sx, sy, seed=pt,
                                                             big_endian=False)
                svc.register_plane(iid, 0, 0, 0, pt, sx, sy, data=data, big_endian=be)
                planes[(pt, be)] = (iid, plane_be)
        ctxs, meta = [], []
        for _ in range(240):
            pt, be = int(rng.integers(8)), bool(rng.integers(2))
            fmt = [None, "png", "tif", "png", "jpeg"][int(rng.integers(5))]
            w, h = int(rng.integers(0, 300)), int(rng.integers(0, 120))
            x, y = int(rng.integers(0, sx - max(w, 1) + 2)), int(rng.integers(0, sy - max(h, 1) + 2))
            ctxs.append(pbx.TileCtx(planes[(pt, be)][0], 0, 0, 0, x, y, w, h, format=fmt))
            meta.append((pt, be, x, y, w, h, fmt))
        res = svc.get_tiles(ctxs)
        ok = 0
        for (pt, be, x, y, w, h, fmt), (st, body) in zip(meta, res):
            fcode = {None: oracle.FMT_RAW, "png": oracle.FMT_PNG, "tif": oracle.FMT_TIF}.get(fmt, oracle.FMT_UNKNOWN)
            plane_be = planes[(pt, be)][1]
            ost, obody, ow, oh = oracle.get_tile(plane_be, True, pt, sx, sy, x, y, w, h, fcode)
            want_status = pbx.OK if ost == 0 else ost
            assert st == want_status, (pt, be, x, y, w, h, fmt, st, ost)
            if st != pbx.OK:
                continue
            ok += 1
            tile = oracle.extract_be(plane_be, True, pt, sx * oracle.BPP[pt], x, y, ow, oh).tobytes()
            if fmt is None:
                assert body == obody == tile
            elif fmt == "tif":
                r, px, m = oracle.tiff_decode(body, len(tile))
                assert r == 0 and px == tile
                if png_filter != pbx.FILTER_ADAPTIVE:   # uncompressed: the oracle's bytes
                    assert body == obody
                else:
                    assert m["compression"] == 8
            else:
                r, px, m = oracle.png_decode(body)
                assert r == 0 and px == _flip(tile, pt)
                stream = oracle.png_filter_stream(np.frombuffer(tile, np.uint8), pt, ow, oh,
                                                  png_filter).tobytes()
                r, idat = oracle.png_inflate_idat(body, len(stream))
                assert r == 0 and idat == stream, (pt, be, x, y, ow, oh)
        assert ok > 60
