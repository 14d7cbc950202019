"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar (BASELINE.json north_star): raw tiles byte-identical; PNG/TIFF decode to bit-exact
pixels.  Stronger checks where they exist: with the reference's filter (None) the
inflated IDAT equals the oracle's filtered scanlines byte for byte, and the GPU's zlib
stream equals the CPU emulation of the same deflate phases (tests/_emu.py) byte for byte.
"""
import itertools
import zlib

import numpy as np
import pytest

import pbx
import _emu

pytestmark = pytest.mark.gpu

_ids = itertools.count(1000)


def host_plane(service, oracle, pt, sx, sy, kind=2, big_endian=True, seed=0):
    """Register an oracle-generated plane from host memory; returns (image_id, plane_be)."""
    iid = next(_ids)
    be = oracle.gen_region(kind, pt, 0, 0, sx, sy, seed=seed, big_endian=True)
    data = be if big_endian else oracle.gen_region(kind, pt, 0, 0, sx, sy, seed=seed,
                                                    big_endian=False)
    service.register_plane(iid, 0, 0, 0, pt, sx, sy, data=data, big_endian=big_endian)
    return iid, be


def oracle_tile(oracle, plane_be, pt, sx, x, y, w, h):
    return oracle.extract_be(plane_be, True, pt, sx * oracle.BPP[pt], x, y, w, h).tobytes()


def flip_png(tile, pt):
    """APNGWriter int8/int16 sign flip of the most significant byte of each sample."""
    a = bytearray(tile)
    if pt in (pbx.INT8, pbx.INT16):
        a[0::pbx.BYTES_PER_PIXEL[pt]] = bytes(b ^ 0x80 for b in a[0::pbx.BYTES_PER_PIXEL[pt]])
    return bytes(a)


# ------------------------------------------------------------------------------ raw

@pytest.mark.parametrize("pt", range(8))
@pytest.mark.parametrize("big_endian", [True, False])
def test_raw_all_types(service, oracle, pt, big_endian):
    sx, sy = 301, 97
    iid, plane = host_plane(service, oracle, pt, sx, sy, big_endian=big_endian)
    regions = [(0, 0, 0, 0), (0, 0, 64, 48), (5, 3, 17, 9), (300, 96, 1, 1), (1, 0, 300, 1),
               (0, 1, 1, 96), (64, 32, 128, 64), (13, 7, 257, 31)]
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, x, y, w, h) for (x, y, w, h) in regions]
    res = service.get_tiles(ctxs)
    for (x, y, w, h), (st, body) in zip(regions, res):
        ww, hh = (w or sx), (h or sy)
        assert st == pbx.OK
        assert body == oracle_tile(oracle, plane, pt, sx, x, y, ww, hh), (pt, x, y, w, h)


def test_generated_planes_match_oracle(service, oracle):
    for kind, gen in ((1, "fake"), (2, "noise")):
        for pt in range(8):
            iid = next(_ids)
            sx, sy = 77, 23
            pid = service.register_plane(iid, 1, 2, 3, pt, sx, sy, generator=gen, seed=5,
                                         plane_no=4)
            got = service.read_plane_be(pid, sx * sy * oracle.BPP[pt])
            want = oracle.gen_region(kind, pt, 0, 0, sx, sy, seed=5, plane_no=4, z=1, c=2, t=3)
            assert got == want.tobytes(), (gen, pt)


# ------------------------------------------------------------------------------ PNG

PNG_TYPES = [pbx.INT8, pbx.UINT8, pbx.INT16, pbx.UINT16]


@pytest.mark.parametrize("pt", PNG_TYPES)
@pytest.mark.parametrize("kind", [1, 2])
def test_png_decodes_bit_exact(png_service, oracle, pt, kind):
    service = png_service
    sx, sy = 700, 333
    iid, plane = host_plane(service, oracle, pt, sx, sy, kind=kind, big_endian=False)
    regions = [(0, 0, 512, 300), (3, 5, 1, 1), (0, 0, 1, 333), (11, 2, 513, 257), (0, 0, 0, 0),
               (699, 0, 1, 7), (100, 100, 64, 48)]
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format="png") for (x, y, w, h) in regions]
    res = service.get_tiles(ctxs)
    for (x, y, w, h), (st, body) in zip(regions, res):
        ww, hh = (w or sx), (h or sy)
        assert st == pbx.OK, (x, y, w, h)
        tile = oracle_tile(oracle, plane, pt, sx, x, y, ww, hh)
        r, px, meta = oracle.png_decode(body)
        assert r == 0, r
        assert (meta["w"], meta["h"], meta["depth"], meta["color_type"]) == (ww, hh, 8 * oracle.BPP[pt], 0)
        assert px == flip_png(tile, pt)
        # filter None (the reference's) -> the inflated IDAT is the oracle's filtered stream
        stream = oracle.png_filter_stream(np.frombuffer(tile, np.uint8), pt, ww, hh, 0).tobytes()
        r, idat = oracle.png_inflate_idat(body, len(stream))
        assert r == 0 and idat == stream
        # and the zlib stream is exactly the CPU emulation of the deflate workgroups
        z, _ = _emu.deflate(stream, 1 + ww * oracle.BPP[pt])
        start = 99
        assert body[start:start + len(z)] == z


@pytest.mark.parametrize("big_endian", [False, True])
@pytest.mark.parametrize("pt", [pbx.UINT16, pbx.INT16, pbx.UINT8])
def test_png_row_shapes(png_service, oracle, pt, big_endian):
    """Row layouts of the direct plane reader and of the banded row kernel: 2 KiB - 8 KiB
    rows (large LDS bands), row lengths that are not multiples of 16, band tails, aligned
    and unaligned starts."""
    service = png_service
    sx, sy = 4200, 41
    iid, plane = host_plane(service, oracle, pt, sx, sy, kind=2, big_endian=big_endian)
    bpp = oracle.BPP[pt]
    regions = [(0, 0, 4096, 20), (0, 1, 2048, 33), (16, 1, 2064, 17), (32, 7, 1000, 34),
               (8, 0, 777, 41), (0, 0, 31, 16), (0, 0, 15, 3), (4192 // bpp, 2, 8, 39)]
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format="png") for (x, y, w, h) in regions]
    res = service.get_tiles(ctxs)
    for (x, y, w, h), (st, body) in zip(regions, res):
        assert st == pbx.OK, (x, y, w, h)
        tile = oracle_tile(oracle, plane, pt, sx, x, y, w, h)
        stream = oracle.png_filter_stream(np.frombuffer(tile, np.uint8), pt, w, h, 0).tobytes()
        r, idat = oracle.png_inflate_idat(body, len(stream))
        assert r == 0 and idat == stream, (pt, x, y, w, h)


@pytest.mark.parametrize("pt", [pbx.INT32, pbx.UINT32, pbx.FLOAT, pbx.DOUBLE])
def test_png_rejects_wide_types(service, oracle, pt):
    iid, _ = host_plane(service, oracle, pt, 40, 30)
    (st, body), = service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, 0, 0, 8, 8, format="png")])
    assert st == pbx.E_NOTFOUND and body is None


def test_png_pil_decodes(service, oracle):
    pytest.importorskip("PIL")
    import io
    from PIL import Image
    iid, plane = host_plane(service, oracle, pbx.UINT16, 600, 520, big_endian=False)
    (st, body), = service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, 40, 4, 512, 512, format="png")])
    assert st == pbx.OK
    im = np.array(Image.open(io.BytesIO(body)))
    want = np.frombuffer(oracle_tile(oracle, plane, pbx.UINT16, 600, 40, 4, 512, 512),
                         ">u2").reshape(512, 512)
    assert (im.astype(np.uint16) == want).all()


# ------------------------------------------------------------------------------ TIFF

@pytest.mark.parametrize("pt", range(8))
def test_tiff_all_types(service, oracle, pt):
    sx, sy = 260, 70
    iid, plane = host_plane(service, oracle, pt, sx, sy, big_endian=(pt % 2 == 0))
    regions = [(0, 0, 0, 0), (3, 1, 5, 7), (16, 8, 128, 32), (0, 0, 1, 1)]
    res = service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, *r, format="tif") for r in regions])
    for (x, y, w, h), (st, body) in zip(regions, res):
        ww, hh = (w or sx), (h or sy)
        assert st == pbx.OK
        r, px, meta = oracle.tiff_decode(body, ww * hh * oracle.BPP[pt])
        assert r == 0, r
        assert meta["big_endian"] == 1 and meta["compression"] == 1
        assert (meta["w"], meta["h"], meta["bits"]) == (ww, hh, 8 * oracle.BPP[pt])
        assert px == oracle_tile(oracle, plane, pt, sx, x, y, ww, hh)
        # uncompressed TIFF is byte-identical to the oracle's writer
        st2, ref = oracle.tiff_encode(np.frombuffer(px, np.uint8), pt, ww, hh)
        assert body == ref


# -------------------------------------------------------------------- error parity

def test_error_statuses(service, oracle):
    iid, _ = host_plane(service, oracle, pbx.UINT16, 50, 40)
    cases = [
        # an image / plane this context does not hold: the binding looks it up and loads it
        # (getPixels + getPixelBuffer); without a PixelSource the handler answers 404 below
        (pbx.TileCtx(iid + 999999, 0, 0, 0), pbx.E_NOT_RESIDENT),             # unknown image
        (pbx.TileCtx(iid, 1, 0, 0, 0, 0, 4, 4), pbx.E_NOT_RESIDENT),          # z not loaded
        (pbx.TileCtx(iid, 0, 0, 0, 48, 0, 4, 4), pbx.E_NOTFOUND),             # out of bounds
        (pbx.TileCtx(iid, 0, 0, 0, -1, 0, 4, 4), pbx.E_NOTFOUND),
        (pbx.TileCtx(iid, 0, 0, 0, 10, 0, 0, 4), pbx.E_NOTFOUND),             # w default + x
        (pbx.TileCtx(iid, 0, 0, 0, 0, 0, 4, 4, format="jpg"), pbx.E_NOTFOUND),  # unknown fmt
        (pbx.TileCtx(iid, 0, 0, 0, 0, 0, 4, 4, resolution=1), pbx.E_NOTFOUND),  # 1 level only
        (pbx.TileCtx(iid, 0, 0, 0, 0, 0, 4, 4, resolution=0), pbx.OK),          # = full res
        (pbx.TileCtx(iid, 0, 0, 0, 0, 0, 4, 4, format="png"), pbx.OK),
        (pbx.TileCtx(iid, 0, 0, 0, 0, 0, 65536, 65536), pbx.E_NOTFOUND),       # int overflow
    ]
    res = service.get_tiles([c for c, _ in cases])
    assert [st for st, _ in res] == [want for _, want in cases]
    # the event-bus consumer mapping (PixelBufferVerticle.java:90-147)
    st, body, hdr = pbx.handle_get_tile(service, "{not json")
    assert st == 400
    for c, _ in cases[:2]:  # closed registry (no PixelSource): not resident -> null -> 404
        st, body, hdr = pbx.handle_get_tile(service, c.to_json())
        assert st == 404 and body == f"Cannot find Image:{c.imageId}".encode()
    ok = pbx.TileCtx(iid, 0, 0, 0, 1, 2, 0, 3)
    st, body, hdr = pbx.handle_get_tile(service, ok.to_json())
    assert st == 404  # w defaults to 50 with x=1 -> outside the plane
    ok = pbx.TileCtx(iid, 0, 0, 0, 0, 2, 0, 3, format="tif")
    st, body, hdr = pbx.handle_get_tile(service, ok.to_json())
    assert st == 200 and hdr["filename"] == f"image{iid}_z0_c0_t0_x0_y2_w50_h3.tif"
    assert hdr["Content-Type"] == "image/tiff"


def test_resolution_levels(service, oracle):
    """OMERO's resolution numbering (TileRequestHandler.java:89-91 -> setResolutionLevel):
    with L stored levels, resolution L-1 is the full-resolution plane and 0 the smallest
    (omero-zarr-pixel-buffer maps it to NGFF dataset L-1-resolution); an absent resolution
    serves full resolution; w/h defaulting uses the full-resolution Pixels size (:92-97);
    a level outside [0, L) -> setResolutionLevel throws -> null -> 404."""
    iid, plane = host_plane(service, oracle, pbx.UINT8, 64, 64)
    lvl1 = oracle.gen_region(1, pbx.UINT8, 0, 0, 32, 32)
    lvl2 = oracle.gen_region(2, pbx.UINT8, 0, 0, 16, 16, seed=9)
    service.register_plane(iid, 0, 0, 0, pbx.UINT8, 32, 32, data=lvl1, level=1)
    service.register_plane(iid, 0, 0, 0, pbx.UINT8, 16, 16, data=lvl2, level=2)
    full = oracle.extract_be(plane, True, pbx.UINT8, 64, 0, 0, 16, 16).tobytes()
    res = service.get_tiles([
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 16, 16, resolution=2),     # L-1: full resolution
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 16, 16),                   # absent: full resolution
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 16, 16, resolution=1),     # stored level 1
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 16, 16, resolution=0),     # smallest (stored 2)
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 0, 0, resolution=2),       # w/h -> 64 x 64, full res
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 0, 0, resolution=1),       # w/h -> 64: outside 32^2
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 4, 4, resolution=3),       # only 3 levels -> 404
        pbx.TileCtx(iid, 0, 0, 0, 0, 0, 4, 4, resolution=-1),      # given negative -> 404
    ])
    st = [s for s, _ in res]
    assert st == [pbx.OK, pbx.OK, pbx.OK, pbx.OK, pbx.OK, pbx.E_NOTFOUND, pbx.E_NOTFOUND,
                  pbx.E_NOTFOUND], st
    assert res[0][1] == full and res[1][1] == full
    assert res[2][1] == oracle.extract_be(lvl1, True, pbx.UINT8, 32, 0, 0, 16, 16).tobytes()
    assert res[3][1] == lvl2.tobytes()
    assert res[4][1] == plane.tobytes()


# ------------------------------------------------------------- adaptive filter / deflate TIFF

@pytest.mark.parametrize("pt", PNG_TYPES)
def test_png_adaptive_filter(adaptive_service, oracle, pt):
    sx, sy = 530, 300
    iid = next(_ids)
    plane = oracle.gen_region(2, pt, 0, 0, sx, sy)
    adaptive_service.register_plane(iid, 0, 0, 0, pt, sx, sy, data=plane, big_endian=True)
    regions = [(0, 0, 512, 256), (7, 9, 100, 33), (0, 0, 1, 1)]
    res = adaptive_service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, *r, format="png") for r in regions])
    for (x, y, w, h), (st, body) in zip(regions, res):
        assert st == pbx.OK
        tile = oracle_tile(oracle, plane, pt, sx, x, y, w, h)
        r, px, _ = oracle.png_decode(body)
        assert r == 0 and px == flip_png(tile, pt)
        stream = oracle.png_filter_stream(np.frombuffer(tile, np.uint8), pt, w, h, 5).tobytes()
        r, idat = oracle.png_inflate_idat(body, len(stream))
        assert idat == stream  # same per-row filter choice as the oracle's heuristic


@pytest.mark.parametrize("pt", range(8))
def test_tiff_deflate(adaptive_service, oracle, pt):
    iid = next(_ids)
    plane = oracle.gen_region(1, pt, 0, 0, 300, 200)
    adaptive_service.register_plane(iid, 0, 0, 0, pt, 300, 200, data=plane, big_endian=True)
    (st, body), = adaptive_service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, 10, 20, 256, 128,
                                                          format="tif")])
    assert st == pbx.OK
    r, px, meta = oracle.tiff_decode(body, 256 * 128 * oracle.BPP[pt])
    assert r == 0 and meta["compression"] == 8
    assert px == oracle_tile(oracle, plane, pt, 300, 10, 20, 256, 128)


# ------------------------------------------------------------------ batches at scale

def test_batch_4096_png_u16_grid(service, oracle):
    """BASELINE configs[1]/metric shape: 4096 tiles of 512x512 uint16 from one plane.

    Every one of the 4096 tiles is pixel-checked: its IDAT is inflated and the scanlines
    must equal the oracle generator's tile (filter bytes 0).  Samples also decode through the
    oracle's PNG decoder (chunks, IHDR)."""
    iid = next(_ids)
    side = 64 * 512
    service.register_plane(iid, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0)
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, (i % 64) * 512, (i // 64) * 512, 512, 512, format="png")
            for i in range(4096)]
    res = service.get_tiles(ctxs)
    assert all(st == pbx.OK for st, _ in res)
    bodies = [b for _, b in res]
    assert oracle.check_png_grid_pixels(bodies, pbx.UINT16, 512, 512, 64, 0) == []
    for i in (0, 1, 63, 64, 2049, 4095):
        r, px, _ = oracle.png_decode(bodies[i])
        assert r == 0 and px == oracle.gen_region(2, pbx.UINT16, (i % 64) * 512, (i // 64) * 512,
                                                  512, 512).tobytes(), i
    # compression ratio close to zlib-6 (~1.34x on G_NOISE)
    assert sum(map(len, bodies)) < 4096 * 524800 / 1.30


def test_mixed_batch(service, oracle):
    """C5-style mixed stream: uint8/int32/float32 planes, png/tif/raw, 404 for png x wide."""
    rng = np.random.default_rng(0)
    planes = {}
    for pt in (pbx.UINT8, pbx.INT32, pbx.FLOAT):
        iid, be = host_plane(service, oracle, pt, 1030, 900, kind=2)
        planes[pt] = (iid, be)
    ctxs, meta = [], []
    for _ in range(200):
        pt = [pbx.UINT8, pbx.INT32, pbx.FLOAT][rng.integers(3)]
        w, h = int(rng.integers(1, 8)) * 128, int(rng.integers(1, 7)) * 128
        x, y = int(rng.integers(0, 1030 - w + 1)), int(rng.integers(0, 900 - h + 1))
        fmt = [None, "png", "tif"][rng.integers(3)]
        ctxs.append(pbx.TileCtx(planes[pt][0], 0, 0, 0, x, y, w, h, format=fmt))
        meta.append((pt, x, y, w, h, fmt))
    res = service.get_tiles(ctxs)
    for (pt, x, y, w, h, fmt), (st, body) in zip(meta, res):
        tile = oracle_tile(oracle, planes[pt][1], pt, 1030, x, y, w, h)
        if fmt == "png" and pt != pbx.UINT8:
            assert st == pbx.E_NOTFOUND
            continue
        assert st == pbx.OK
        if fmt is None:
            assert body == tile
        elif fmt == "tif":
            r, px, _ = oracle.tiff_decode(body, len(tile))
            assert r == 0 and px == tile
        else:
            r, px, _ = oracle.png_decode(body)
            assert r == 0 and px == tile


def test_tiff_deflate_segment_capacity(adaptive_service):
    """A Huffman block (BLK_SEGS segments) whose code would give one segment more than
    16 KiB of bits is stored (k_huff's seg_shares_fit): the GPU stream equals the CPU
    emulation byte for byte and decodes exactly."""
    from test_emu_deflate import skewed_block_stream
    data = skewed_block_stream()
    w = next(w for w in (256, 1023, 1024, 2048) if len(data) % w == 0)
    h = len(data) // w
    iid = next(_ids)
    plane = np.frombuffer(data, np.uint8).reshape(h, w)
    adaptive_service.register_plane(iid, 0, 0, 0, pbx.UINT8, w, h, data=plane, big_endian=True)
    (st, body), = adaptive_service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, 0, 0, w, h, format="tif")])
    assert st == pbx.OK
    z, blks = _emu.deflate(data, w)
    assert blks[0].btype == 0
    assert body[160:] == z
    assert zlib.decompress(body[160:]) == data


@pytest.mark.parametrize("filt", [pbx.FILTER_SUB, pbx.FILTER_UP, pbx.FILTER_AVG, pbx.FILTER_PAETH,
                                  pbx.FILTER_ADAPTIVE])
def test_png_filters_dword_path(oracle, filt):
    """Filtered PNG rows of whole dwords from aligned source rows go through k_filter2 (SWAR
    filter arithmetic); the inflated IDAT must equal the oracle's filtered scanlines (the
    adaptive choice included) for every PNG type, down to 16-byte and up to 2 KiB rows."""
    with pbx.PixelsService(png_filter=filt) as svc:
        for pt in PNG_TYPES:
            bpp = oracle.BPP[pt]
            sx, sy = 2600 // bpp, 90
            iid = next(_ids)
            plane = oracle.gen_region(2, pt, 0, 0, sx, sy)
            svc.register_plane(iid, 0, 0, 0, pt, sx, sy, data=plane, big_endian=True)
            regions = [(0, 0, 512 // bpp, 40), (16 // bpp, 3, 64 // bpp, 37), (0, 0, 16 // bpp, 5),
                       (32 // bpp, 1, 2048 // bpp, 17), (0, 7, 1024 // bpp, 1)]
            res = svc.get_tiles([pbx.TileCtx(iid, 0, 0, 0, *r, format="png") for r in regions])
            for (x, y, w, h), (st, body) in zip(regions, res):
                assert st == pbx.OK
                tile = oracle_tile(oracle, plane, pt, sx, x, y, w, h)
                r, px, _ = oracle.png_decode(body)
                assert r == 0 and px == flip_png(tile, pt), (pt, x, y, w, h)
                stream = oracle.png_filter_stream(np.frombuffer(tile, np.uint8), pt, w, h, filt).tobytes()
                r, idat = oracle.png_inflate_idat(body, len(stream))
                assert idat == stream, (pt, x, y, w, h)


def test_incompressible_tiles_stored_per_segment(service, adaptive_service, oracle):
    """Random bytes: every Huffman block (up to BLK_SEGS segments) is stored, one stored block per
    segment (a block may then hold more than one stored block's 65535 bytes).  PNG and
    deflate-TIFF tiles of 1024^2 uint8 decode exactly and equal the CPU emulation byte for
    byte."""
    rng = np.random.default_rng(77)
    plane = rng.integers(0, 256, (1100, 1100), dtype=np.uint8)
    iid = next(_ids)
    for s_ in (service, adaptive_service):
        s_.register_plane(iid, 0, 0, 0, pbx.UINT8, 1100, 1100, data=plane, big_endian=True)
    (st, png), = service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, 7, 9, 1024, 1024, format="png")])
    (st2, tif), = adaptive_service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, 7, 9, 1024, 1024, format="tif")])
    assert st == pbx.OK and st2 == pbx.OK
    tile = plane[9:9 + 1024, 7:7 + 1024]
    r, px, _ = oracle.png_decode(png)
    assert r == 0 and px == tile.tobytes()
    stream = np.concatenate([np.zeros((1024, 1), np.uint8), tile], 1).tobytes()
    z, blks = _emu.deflate(stream, 1025)
    assert all(b.btype == 0 for b in blks) and len(blks) > 1
    assert png[99:99 + len(z)] == z
    assert zlib.decompress(z) == stream
    r, px, meta = oracle.tiff_decode(tif, 1024 * 1024)
    assert r == 0 and meta["compression"] == 8 and px == tile.tobytes()
    z2, _ = _emu.deflate(tile.tobytes(), 1024)
    assert tif[160:160 + len(z2)] == z2


@pytest.mark.parametrize("origin", [(0, 0), (1024, 3072), (7680, 512), (13, 7)])
def test_fake_u16_tiles_cross_wave_matches(service, oracle, origin):
    """512x512 uint16 G_FAKE tiles (rows repeating: matches run across the waves' 2 KiB
    sub-segments, and every boundary of a segment takes a carry round): the zlib stream is
    the CPU emulation of the deflate workgroups byte for byte, it inflates to the oracle's
    scanlines, and it stays within 3% of zlib-6."""
    iid = next(_ids)
    service.register_plane(iid, 0, 0, 0, pbx.UINT16, 8192, 4096, generator="fake")
    x, y = origin
    (st, body), = service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, x, y, 512, 512, format="png")])
    assert st == pbx.OK
    tile = oracle.gen_region(1, pbx.UINT16, x, y, 512, 512)
    stream = oracle.png_filter_stream(tile, pbx.UINT16, 512, 512, 0).tobytes()
    r, idat = oracle.png_inflate_idat(body, len(stream))
    assert r == 0 and idat == stream
    z, _ = _emu.deflate(stream, 1025)
    assert body[99:99 + len(z)] == z
    assert len(z) <= 1.03 * len(zlib.compress(stream, 6)) + 64
    service.release_plane(service.lookup_plane(iid, 0, 0, 0)[0])
