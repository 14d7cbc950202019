"""Pixel parity of the deflate chain at the scale the bench runs it.

k_huff has two forms: batches of at most HUFF_SMALL_BLKS = 256 Huffman blocks take the
latency form (every segment's histogram in registers), larger ones the batch form
(kernels_deflate.hip:2077,3443-3454).  Tiles of more than 64 segments are split into
several blocks, and a block boundary inside a tile brings an empty stored block, byte
alignment and a shared-byte hand-off to k_frame.  These tests run exactly the bench's
large-batch workloads through the C-ABI and check EVERY tile (or a seeded sample of a
whole-slide pass) against the CPU oracle (oracle/pbx_oracle.c, the checker only):

* configs[2]: the 4096 x 1024^2 uint16 PNG tiles of the 65536^2 plane, in batches of 1024
  tiles (129 segments = 3 Huffman blocks per tile, 3,072 blocks per launch); every IDAT
  inflated and compared with the oracle generator's big-endian tile
  (TileRequestHandler.java:119-124,176-199; BASELINE configs[2]);
* the adaptive PNG filter (blocks of at most 16 segments: 3 per 512^2 uint16 tile, 12,288 per
  launch) on the headline's 4096-tile batch, G_NOISE and G_FAKE: every tile's inflated IDAT
  equals the oracle's adaptive scanlines (png_filter_stream);
* configs[3] with Compression=8 (the tiff_deflate option): two of the whole-slide pass's own
  batches (49 tile rows x 196 tiles = 9,604 tiles, one block per tile) of a 100000^2 uint16
  channel, the first rows and the last rows (160-px edge tiles), a seeded sample of 512 tiles
  decoded by the oracle's TIFF decoder and compared with the generator's tile.
"""
import numpy as np
import pytest
from concurrent.futures import ThreadPoolExecutor

import pbx

pytestmark = pytest.mark.gpu

NOISE, FAKE = 2, 1
HUFF_SMALL_BLKS = 256


def _run(svc, ctxs):
    """One device-resident batch (the bench's form): plan, launch, sync; (stats, bodies)."""
    b = pbx.Batch(svc, ctxs)
    try:
        b.launch()
        b.sync()
        st = b.stats()
        res = b.fetch()
    finally:
        b.close()
    assert all(s == pbx.OK for s, _ in res)
    return st, [body for _, body in res]


def test_c3_png_4096x1024x1024_u16_every_tile(oracle):
    """configs[2] exactly: 4096 1024^2 uint16 PNG tiles of the 65536^2 G_NOISE plane, four
    launches of 1024 tiles (> 256 Huffman blocks each), every tile pixel-checked."""
    side, T, G, per = 65536, 1024, 64, 1024
    with pbx.PixelsService() as svc:
        svc.register_plane(3, 0, 0, 0, pbx.UINT16, side, side, generator="noise")
        for k in range(G * G // per):
            ctxs = [pbx.TileCtx(3, 0, 0, 0, (i % G) * T, (i // G) * T, T, T, format="png")
                    for i in range(k * per, (k + 1) * per)]
            st, bodies = _run(svc, ctxs)
            assert st.png_tiles == per and st.segments >= per * 129
            assert st.blocks >= per * 3 and st.blocks > HUFF_SMALL_BLKS  # multi-block tiles
            bad = oracle.check_png_grid_pixels(bodies, pbx.UINT16, T, T, G, (k * per // G) * T,
                                               threads=16)
            assert bad == [], (k, bad[:8])


@pytest.mark.parametrize("gen", ["noise", "fake"])
def test_adaptive_filter_4096_tiles_every_tile(oracle, gen):
    """The headline batch (4096 x 512^2 uint16 of the 32768^2 plane) through the adaptive
    filter: three Huffman blocks per tile (12,288 per launch); every tile's IDAT inflates to the
    oracle's adaptive scanlines."""
    side, T, G = 32768, 512, 64
    kind = NOISE if gen == "noise" else FAKE
    with pbx.PixelsService(png_filter=pbx.FILTER_ADAPTIVE) as svc:
        svc.register_plane(4, 0, 0, 0, pbx.UINT16, side, side, generator=gen)
        ctxs = [pbx.TileCtx(4, 0, 0, 0, (i % G) * T, (i // G) * T, T, T, format="png")
                for i in range(G * G)]
        st, bodies = _run(svc, ctxs)
    assert st.blocks >= G * G * 3 and st.blocks > HUFF_SMALL_BLKS  # multi-block tiles
    cap = T * (1 + 2 * T)

    def row(r):
        band = oracle.gen_region(kind, pbx.UINT16, 0, r * T, side, T).reshape(T, side * 2)
        bad = []
        for x in range(G):
            tile = np.ascontiguousarray(band[:, x * T * 2:(x + 1) * T * 2]).reshape(-1)
            want = oracle.png_filter_stream(tile, pbx.UINT16, T, T, pbx.FILTER_ADAPTIVE).tobytes()
            rc, idat = oracle.png_inflate_idat(bodies[r * G + x], cap)
            if rc != 0 or idat != want:
                bad.append(r * G + x)
        return bad

    with ThreadPoolExecutor(16) as ex:
        bad = [i for part in ex.map(row, range(G)) for i in part]
    assert bad == [], bad[:8]


def test_wholeslide_deflate_tiff_pass_sample(oracle):
    """configs[3] with Compression=8: the whole-slide pass's first and last batches of a
    100000^2 uint16 channel (9,604 tiles each, as bench.wholeslide_line cuts them), a seeded
    sample of 512 of their tiles decoded by the oracle and compared with the generator."""
    side, T, rows_per = 100000, 512, 49
    n = (side + T - 1) // T
    rng = np.random.default_rng(606)
    with pbx.PixelsService(tiff_deflate=True) as svc:
        checks = []
        for c, r0 in ((0, 0), (4, n - rows_per)):
            svc.register_plane(6, 0, c, 0, pbx.UINT16, side, side, generator="noise", plane_no=c)
            ctxs = [pbx.TileCtx(6, 0, c, 0, T * tx, T * ty, min(T, side - T * tx), min(T, side - T * ty),
                                format="tif") for ty in range(r0, r0 + rows_per) for tx in range(n)]
            st, bodies = _run(svc, ctxs)
            assert st.tiles == rows_per * n and st.blocks > HUFF_SMALL_BLKS
            pick = rng.choice(len(ctxs), 256, replace=False)
            if r0:  # the corner tile (160 x 160) and the last row's first tile always
                pick = np.unique(np.concatenate([pick, [len(ctxs) - 1, len(ctxs) - n]]))
            checks += [(c, ctxs[i].x, ctxs[i].y, ctxs[i].w, ctxs[i].h, bodies[i]) for i in pick]
            del bodies

    def one(a):
        c, x, y, w, h, body = a
        tile = oracle.gen_region(NOISE, pbx.UINT16, x, y, w, h, plane_no=c, c=c).tobytes()
        r, px, meta = oracle.tiff_decode(body, len(tile))
        return r == 0 and meta["compression"] == 8 and (meta["w"], meta["h"]) == (w, h) and px == tile

    with ThreadPoolExecutor(16) as ex:
        ok = list(ex.map(one, checks))
    assert len(checks) >= 512
    assert all(ok), [checks[i][:5] for i, v in enumerate(ok) if not v][:8]
    assert any(a[3] == 160 and a[4] == 160 for a in checks)


def test_adaptive_tile_mode_poisson(oracle):
    """The adaptive filter's tile mode (k_adaptive_mode, kernels_io.hip) on a
    Poisson-like uint16 plane (microscope counts, lambda drifting 200..300, the bench's
    adaptive_filter_line plane) and on G_FAKE: regions that go to k_filter3 (rows of 16-byte
    chunks), k_filter2 (rows of dwords) and the banded k_filter (odd x or odd widths) in one
    batch, every IDAT equal to the oracle's adaptive scanlines, the None-mode tiles exactly the
    oracle's (adaptive_tile_none), and the 64 whole 512^2 Poisson tiles no larger in total than
    the same tiles through filter None."""
    side, T = 4096, 512
    rng = np.random.default_rng(1234)
    yy, xx = np.mgrid[0:side:64, 0:side:64]
    lam = 200.0 + 100.0 * (0.5 + 0.25 * np.sin(xx / 900.0) + 0.25 * np.cos(yy / 1300.0))
    pois = rng.poisson(np.repeat(np.repeat(lam, 64, 0), 64, 1)).astype(np.uint16)
    pois_be = pois.astype(">u2").view(np.uint8).reshape(side, side * 2)
    fake_be = oracle.gen_region(FAKE, pbx.UINT16, 0, 0, side, 64).reshape(64, side * 2)
    regions = [(0, (i % 8) * T, (i // 8) * T, T, T) for i in range(64)]  # k_filter3
    for k in range(96):
        w = int(rng.choice([8, 24, 40, 136, 250, 1030, 1001]))  # 16 B chunks, dwords, odd
        h = int(rng.integers(1, 61))
        x = int(rng.integers(0, side - w)) & ~(7 if k % 3 else 0)
        y = int(rng.integers(0, 64 - h + 1)) if k % 4 == 0 else int(rng.integers(0, side - h))
        regions.append((1 if k % 4 == 0 else 0, x, y, w, h))
    with pbx.PixelsService(png_filter=pbx.FILTER_ADAPTIVE) as sa, pbx.PixelsService() as sn:
        for s_ in (sa, sn):
            s_.register_plane(7, 0, 0, 0, pbx.UINT16, side, side, data=pois, big_endian=False)
            s_.register_plane(8, 0, 0, 0, pbx.UINT16, side, side, generator="fake")
        ctxs = [pbx.TileCtx(7 + p, 0, 0, 0, x, y, w, h, format="png") for p, x, y, w, h in regions]
        st_ad, ad = _run(sa, ctxs)
        _, no = _run(sn, ctxs[:64])
    n_none = 0
    for (p, x, y, w, h), body in zip(regions, ad):
        src = pois_be if p == 0 else fake_be
        tile = np.ascontiguousarray(src[y:y + h, 2 * x:2 * (x + w)]).reshape(-1)
        want = oracle.png_filter_stream(tile, pbx.UINT16, w, h, pbx.FILTER_ADAPTIVE).tobytes()
        rc, idat = oracle.png_inflate_idat(body, len(want))
        assert rc == 0 and idat == want, (p, x, y, w, h)
        mode = oracle.adaptive_tile_none(tile, pbx.UINT16, w, h)
        filt = np.frombuffer(idat, np.uint8).reshape(h, 1 + 2 * w)[:, 0]
        assert not mode or not filt.any(), (p, x, y, w, h)
        n_none += mode
    assert n_none >= 64  # every whole Poisson tile, at least
    # None-mode tiles of TF_DIRECT's geometry (the 64 whole tiles among them) skip the filter
    # pass: k_lz77 reads their rows from the plane
    assert 64 <= st_ad.direct_tiles <= n_none
    assert sum(map(len, ad[:64])) <= sum(map(len, no))


@pytest.mark.parametrize("pt", [pbx.INT8, pbx.UINT8, pbx.INT16, pbx.UINT16])
def test_adaptive_tile_mode_types_and_small_shapes(oracle, pt):
    """The tile mode on every PNG pixel type (the int8 / int16 sign flip comes before the mode's
    byte counts) and on small shapes: one row (the middle row's prediction row is zeros above
    the tile), one or two samples per row, rows of one 16-byte chunk; Poisson-like counts
    around a per-type offset and G_FAKE side by side in one batch, every IDAT equal to the
    oracle's adaptive scanlines and the None-mode tiles exactly the oracle's."""
    side = 1024
    bpp = oracle.BPP[pt]
    rng = np.random.default_rng(90 + pt)
    lam = 20.0 if bpp == 1 else 300.0
    dt = {pbx.INT8: "i1", pbx.UINT8: "u1", pbx.INT16: ">i2", pbx.UINT16: ">u2"}[pt]
    base = -60 if pt == pbx.INT8 else 0 if bpp == 1 else -2000 if pt == pbx.INT16 else 1000
    pois = (rng.poisson(lam, (side, side)) + base).astype(dt)
    pois_be = np.frombuffer(pois.tobytes(), np.uint8).reshape(side, side * bpp)
    fake_be = oracle.gen_region(FAKE, pt, 0, 0, side, side).reshape(side, side * bpp)
    shapes = [(1, 1), (2, 1), (3, 2), (1, 7), (16 // bpp, 1), (16 // bpp, 5), (33, 1), (64, 64),
              (100, 3), (257, 9), (512, 40), (1000, 2)]
    regions = []
    for k, (w, h) in enumerate(shapes * 2):
        p = k % 2
        x = int(rng.integers(0, side - w)) & (~15 if k % 3 else ~0)
        y = int(rng.integers(0, side - h))
        regions.append((p, x, y, w, h))
    with pbx.PixelsService(png_filter=pbx.FILTER_ADAPTIVE) as svc:
        svc.register_plane(9, 0, 0, 0, pt, side, side, data=pois_be.reshape(-1), big_endian=True)
        svc.register_plane(10, 0, 0, 0, pt, side, side, generator="fake")
        ctxs = [pbx.TileCtx(9 + p, 0, 0, 0, x, y, w, h, format="png") for p, x, y, w, h in regions]
        _, bodies = _run(svc, ctxs)
    modes = []
    for (p, x, y, w, h), body in zip(regions, bodies):
        src = pois_be if p == 0 else fake_be
        tile = np.ascontiguousarray(src[y:y + h, bpp * x:bpp * (x + w)]).reshape(-1)
        want = oracle.png_filter_stream(tile, pt, w, h, pbx.FILTER_ADAPTIVE).tobytes()
        rc, idat = oracle.png_inflate_idat(body, len(want))
        assert rc == 0 and idat == want, (p, x, y, w, h)
        modes.append(oracle.adaptive_tile_none(tile, pt, w, h))
    assert any(modes) and not all(modes)
