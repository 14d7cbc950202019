"""GPU parity for the BASELINE.json configs beyond the headline, and the serving path.

* configs[2] (C3): 1024x1024 uint16 PNG tiles;
* configs[3] (C4): whole-slide, multi-channel uint16, every tile as TIFF, tile-row bands
  per rank, edge tiles narrower than 512;
* configs[4] (C5): mixed uint8/int32/float32 stream, 256..2048-px tiles, png/tif/raw;
* the request coalescer behind pbx_get_tile (many concurrent callers, one batch per
  GPU-busy interval) and the D2H copy stream.

Everything goes through the C-ABI (libpbx.so); the oracle (oracle/pbx_oracle.c) is the
checker only.
"""
import itertools
import threading
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import pbx

pytestmark = pytest.mark.gpu

_ids = itertools.count(5000)


def _oracle_tile(oracle, kind, pt, x, y, w, h, c=0, plane_no=0):
    return oracle.gen_region(kind, pt, x, y, w, h, plane_no=plane_no, c=c).tobytes()


def test_c3_png_1024_u16(service, oracle):
    """configs[2] shape: 1024x1024 uint16 PNG tiles from a generated plane (64 tiles of an
    8192^2 plane); every tile decodes bit-exact to the oracle's pixels, and the IDAT of one
    equals the oracle's filter-None scanlines."""
    iid = next(_ids)
    side = 8192
    service.register_plane(iid, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0)
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, (i % 8) * 1024, (i // 8) * 1024, 1024, 1024,
                        format="png") for i in range(64)]
    res = service.get_tiles(ctxs)
    assert all(st == pbx.OK for st, _ in res)
    for i, (_, body) in enumerate(res):
        x, y = (i % 8) * 1024, (i // 8) * 1024
        tile = _oracle_tile(oracle, 2, pbx.UINT16, x, y, 1024, 1024)
        r, px, _ = oracle.png_decode(body)
        assert r == 0 and px == tile, i
    tile = oracle.gen_region(2, pbx.UINT16, 0, 0, 1024, 1024)
    want = oracle.png_filter_stream(tile, pbx.UINT16, 1024, 1024, 0).tobytes()
    r, raw = oracle.png_inflate_idat(res[0][1], len(want))
    assert r == 0 and raw == want
    # compressed size within 1% of zlib level 6 (ImageIO) on the same stream
    assert len(res[0][1]) < 1.01 * len(zlib.compress(want, 6)) + 200


@pytest.mark.parametrize("world", [1, 2, 3])
def test_c4_wholeslide_tiff_bands(service, oracle, world):
    """configs[3] shape, scaled: a 5-channel uint16 slide whose size is not a multiple of
    512 (edge tiles 160 px, as 100000 = 195*512 + 160), every tile as TIFF; each rank
    serves its contiguous band of tile rows.  The bands partition the grid, and every
    TIFF equals the oracle's TIFF of the same tile byte for byte."""
    iid = next(_ids)
    side = 3 * 512 + 160
    ntile = 4
    for c in range(5):
        service.register_plane(iid, 0, c, 0, pbx.UINT16, side, side, generator="noise",
                               seed=0, plane_no=c)
    seen = set()
    for rank in range(world):
        lo, hi = pbx.band_rows(ntile, world, rank)
        ctxs, keys = [], []
        for c in range(5):
            for ty in range(lo, hi):
                for tx in range(ntile):
                    w = min(512, side - 512 * tx)
                    h = min(512, side - 512 * ty)
                    ctxs.append(pbx.TileCtx(iid, 0, c, 0, 512 * tx, 512 * ty, w, h,
                                            format="tif"))
                    keys.append((c, tx, ty, w, h))
        res = service.get_tiles(ctxs)
        for (c, tx, ty, w, h), (st, body) in zip(keys, res):
            assert st == pbx.OK
            assert (c, tx, ty) not in seen
            seen.add((c, tx, ty))
            tile = oracle.gen_region(2, pbx.UINT16, 512 * tx, 512 * ty, w, h, plane_no=c, c=c)
            assert body == oracle.tiff_encode(tile, pbx.UINT16, w, h)[1], (c, tx, ty)
    assert len(seen) == 5 * ntile * ntile


def test_c5_mixed_stream_full_sizes(service, oracle):
    """configs[4] shape: uint8/int32/float32 planes; w,h in {256, 512, ..., 2048};
    png/tif/raw uniformly; PNG of int32/float32 -> 404 (APNGWriter rejects them)."""
    rng = np.random.default_rng(7)
    side = 4096
    planes = {}
    for pt in (pbx.UINT8, pbx.INT32, pbx.FLOAT):
        iid = next(_ids)
        service.register_plane(iid, 0, 0, 0, pt, side, side, generator="noise", seed=0)
        planes[pt] = iid
    ctxs, meta = [], []
    for _ in range(96):
        pt = [pbx.UINT8, pbx.INT32, pbx.FLOAT][rng.integers(3)]
        w, h = int(rng.integers(1, 9)) * 256, int(rng.integers(1, 9)) * 256
        x, y = int(rng.integers(0, side - w + 1)), int(rng.integers(0, side - h + 1))
        fmt = [None, "png", "tif"][rng.integers(3)]
        ctxs.append(pbx.TileCtx(planes[pt], 0, 0, 0, x, y, w, h, format=fmt))
        meta.append((pt, x, y, w, h, fmt))
    res = service.get_tiles(ctxs)
    for k, ((pt, x, y, w, h, fmt), (st, body)) in enumerate(zip(meta, res)):
        if fmt == "png" and pt != pbx.UINT8:
            assert st == pbx.E_NOTFOUND
            continue
        assert st == pbx.OK
        tile = _oracle_tile(oracle, 2, pt, x, y, w, h)
        if fmt is None:
            assert body == tile, k
        elif fmt == "tif":
            want = oracle.tiff_encode(np.frombuffer(tile, np.uint8).copy(), pt, w, h)[1]
            assert body == want, k
        else:
            r, px, _ = oracle.png_decode(body)
            assert r == 0 and px == tile, k


def _check_result(oracle, pt, ctx, st, body):
    x, y, w, h, fmt = ctx.x, ctx.y, ctx.w, ctx.h, ctx.format
    if fmt == "bmp":
        assert st == pbx.E_NOTFOUND and body is None
        return
    assert st == pbx.OK
    tile = _oracle_tile(oracle, 2, pt, x, y, w, h)
    if fmt is None:
        assert body == tile
    elif fmt == "tif":
        r, px, _ = oracle.tiff_decode(body, len(tile))
        assert r == 0 and px == tile
    else:
        r, px, _ = oracle.png_decode(body)
        assert r == 0 and px == tile


@pytest.mark.parametrize("coalesce", [True, False])
def test_concurrent_get_tile(oracle, coalesce):
    """Vert.x-style serving: 32 threads each call pbx_get_tile (TileRequestHandler.getTile)
    for their own requests.  With coalescing, requests arriving while the GPU is busy share
    a batch (fewer batches than requests); every response is still exactly its own tile,
    and a bad request (unknown format -> 404) does not disturb its batch-mates."""
    with pbx.PixelsService(coalesce=coalesce) as svc:
        iid = next(_ids)
        side = 2048
        svc.register_plane(iid, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0)
        rng = np.random.default_rng(3)
        ctxs = []
        for i in range(384):
            w, h = int(rng.integers(1, 5)) * 128, int(rng.integers(1, 5)) * 128
            x, y = int(rng.integers(0, side - w + 1)), int(rng.integers(0, side - h + 1))
            fmt = [None, "png", "tif", "bmp"][i % 4] if i % 17 == 0 else ["png", None, "tif"][i % 3]
            ctxs.append(pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format=fmt))
        b0, r0 = svc.ctx_stats()
        errors = []
        barrier = threading.Barrier(32)

        def worker(k):
            barrier.wait()
            for j in range(k, len(ctxs), 32):
                try:
                    st, body = svc.get_tile(ctxs[j])
                    _check_result(oracle, pbx.UINT16, ctxs[j], st, body)
                except AssertionError as e:  # report, don't hang the pool
                    errors.append((j, repr(e)))

        with ThreadPoolExecutor(32) as ex:
            list(ex.map(worker, range(32)))
        assert not errors, errors[:3]
        b1, r1 = svc.ctx_stats()
        assert r1 - r0 == len(ctxs)
        if coalesce:
            assert b1 - b0 < len(ctxs)
        else:
            assert b1 - b0 == len(ctxs)
        # the reference's single-request handler mirror goes through the same path
        h = pbx.TileRequestHandler(svc, pbx.TileCtx(iid, 0, 0, 0, 0, 0, 64, 64))
        assert h.get_tile() == _oracle_tile(oracle, 2, pbx.UINT16, 0, 0, 64, 64)
        assert pbx.TileRequestHandler(svc, pbx.TileCtx(iid, 0, 0, 0, side, 0, 64, 64)).get_tile() is None


def test_pipelined_batches_overlap_d2h(service, oracle):
    """Batches launched back to back, each fetched (D2H on the copy stream) while the next
    one runs: every fetch returns its own batch's bytes."""
    iid = next(_ids)
    service.register_plane(iid, 0, 0, 0, pbx.UINT16, 4096, 4096, generator="noise", seed=1)
    batches = []
    for k in range(4):
        ctxs = [pbx.TileCtx(iid, 0, 0, 0, 512 * ((i + k) % 8), 512 * ((i // 8 + k) % 8), 512, 512,
                            format="png" if k % 2 == 0 else None) for i in range(64)]
        b = pbx.Batch(service, ctxs)
        b.launch()
        batches.append((ctxs, b))
    for ctxs, b in batches:
        res = b.fetch()
        b.close()
        for i in (0, 17, 63):
            c = ctxs[i]
            tile = oracle.gen_region(2, pbx.UINT16, c.x, c.y, 512, 512, seed=1).tobytes()
            st, body = res[i]
            assert st == pbx.OK
            if c.format is None:
                assert body == tile
            else:
                r, px, _ = oracle.png_decode(body)
                assert r == 0 and px == tile


def test_submit_wait(service, oracle):
    """Batched async C-ABI (pbx_submit / pbx_wait): several batches in flight,
    polled with a zero timeout and collected out of order; each returns its own tiles, and
    a bad request fails alone with the reference's 404."""
    iid = next(_ids)
    service.register_plane(iid, 0, 0, 0, pbx.UINT16, 2048, 2048, generator="noise", seed=3)
    sets = []
    for k in range(3):
        ctxs = [pbx.TileCtx(iid, 0, 0, 0, 256 * ((i + k) % 8), 256 * (i // 8), 256, 256,
                            format=("png", None, "tif")[k]) for i in range(32)]
        ctxs.append(pbx.TileCtx(iid, 0, 0, 0, 2000, 0, 256, 256))  # out of bounds -> 404
        sets.append((ctxs, service.submit(ctxs)))
    first = sets[0][1].wait(0)  # a poll: the results, or None while the batch runs
    got = {0: first} if first is not None else {}
    for k in (2, 1, 0):
        if k not in got:
            got[k] = sets[k][1].wait()
    for k, (ctxs, t) in enumerate(sets):
        res = got[k]
        assert len(res) == len(ctxs)
        assert res[-1] == (pbx.E_NOTFOUND, None)
        for i in (0, 9, 31):
            c = ctxs[i]
            tile = oracle.gen_region(2, pbx.UINT16, c.x, c.y, 256, 256, seed=3).tobytes()
            st, body = res[i]
            assert st == pbx.OK
            if k == 0:
                r, px, _ = oracle.png_decode(body)
            elif k == 1:
                r, px = 0, body
            else:
                r, px, _ = oracle.tiff_decode(body, len(tile))
            assert r == 0 and px == tile, (k, i)
        with pytest.raises(RuntimeError):
            t.wait()


@pytest.mark.parametrize("pt", range(8))
@pytest.mark.parametrize("source", ["host_be", "gen"])
def test_resolution_pyramid(service, oracle, pt, source):
    """On-GPU resolution pyramid (row f3): every level equals the numpy restatement of the
    2x2 box mean applied level by level (bit-exact, floats included), and tiles of a level
    are served through the ordinary getTile path with `resolution` (raw and PNG)."""
    import _numpy_ref as R
    iid = next(_ids)
    sx, sy = 301, 97
    dt = R.DTYPES_BE[pt]
    be = oracle.gen_region(2, pt, 0, 0, sx, sy, seed=7)
    if source == "host_be":
        pid = service.register_plane(iid, 0, 0, 0, pt, sx, sy, data=be, big_endian=True)
    else:
        pid = service.register_plane(iid, 0, 0, 0, pt, sx, sy, generator="noise", seed=7)
    ids = service.build_pyramid(pid, 4)
    want = want0 = np.frombuffer(be.tobytes(), dt).reshape(sy, sx)
    for k, lid in enumerate(ids, start=1):
        want = R.downsample(want)
        h, w = want.shape
        got = service.read_plane_be(lid, w * h * oracle.BPP[pt])
        assert got == want.astype(dt).tobytes(), (pt, source, k)
    # tiles of stored level 2 (76 x 25) = OMERO resolution 5-1-2 = 2 of the 5 levels: raw
    # bytes and (8/16-bit types) PNG pixels; resolution 4 = the full-resolution plane
    lvl = R.downsample(R.downsample(np.frombuffer(be.tobytes(), dt).reshape(sy, sx))).astype(dt)
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, 3, 2, 40, 20, resolution=2),
            pbx.TileCtx(iid, 0, 0, 0, 0, 0, 76, 25, resolution=2, format="png"),
            pbx.TileCtx(iid, 0, 0, 0, 70, 20, 10, 10, resolution=2),  # past the level -> 404
            pbx.TileCtx(iid, 0, 0, 0, 3, 2, 40, 20, resolution=4),
            pbx.TileCtx(iid, 0, 0, 0, 0, 0, 19, 7, resolution=0)]     # stored level 4: 19 x 7
    (s1, raw), (s2, png), (s3, _), (s4, full), (s5, small) = service.get_tiles(ctxs)
    assert s1 == pbx.OK and raw == lvl[2:22, 3:43].tobytes()
    assert s3 == pbx.E_NOTFOUND
    assert s4 == pbx.OK and full == want0[2:22, 3:43].astype(dt).tobytes()
    assert s5 == pbx.OK and small == want.astype(dt).tobytes()  # the smallest level, whole
    if pt in (pbx.INT8, pbx.UINT8, pbx.INT16, pbx.UINT16):
        assert s2 == pbx.OK
        r, px, _ = oracle.png_decode(png)
        bpp = oracle.BPP[pt]
        flip = bytearray(lvl.tobytes())
        if pt in (pbx.INT8, pbx.INT16):
            flip[0::bpp] = bytes(b ^ 0x80 for b in flip[0::bpp])
        assert r == 0 and px == bytes(flip)
    else:
        assert s2 == pbx.E_NOTFOUND  # APNGWriter rejects 32/64-bit types


@pytest.mark.parametrize("streams,stagger", [(3, 1), (2, 0), (4, 2), (3, 4)])
def test_kernel_streams_overlap_same_bytes(service, streams, stagger):
    """Pipelined batches overlapped on several kernel streams (pbx_set_kernel_streams), each
    staggered behind the previous batch's stage, return exactly the bytes the same batches
    give one at a time on one stream (PNG and deflate-free batches interleaved)."""
    iid = next(_ids)
    service.register_plane(iid, 0, 0, 0, pbx.UINT16, 4096, 4096, generator="noise", seed=5)

    def run(ns, sg):
        service.set_kernel_streams(ns, sg)
        out = []
        try:
            batches = []
            for k in range(6):
                ctxs = [pbx.TileCtx(iid, 0, 0, 0, 512 * ((i + k) % 8), 512 * ((i // 8 + k) % 8), 512, 512,
                                    format=None if k == 3 else "png") for i in range(64)]
                b = pbx.Batch(service, ctxs)
                b.launch()
                batches.append(b)
            for b in batches:
                out.append(b.fetch())
                b.close()
        finally:
            service.set_kernel_streams(3, 1)
        return out

    want = run(1, 0)
    got = run(streams, stagger)
    assert got == want


def test_kernel_streams_bad_arguments(service):
    """pbx_set_kernel_streams: 1..4 streams, stagger 0..4; anything else is a 400 and keeps
    the setting."""
    for ns, sg in [(0, 1), (5, 1), (3, -1), (3, 5)]:
        with pytest.raises(pbx.PbxError) as e:
            service.set_kernel_streams(ns, sg)
        assert e.value.status == pbx.E_BADARG
    service.set_kernel_streams(3, 1)
