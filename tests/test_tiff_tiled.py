"""Tiled TIFF: `cfg.tiff_tile = T` answers `format=tif` with a TIFF 6.0
tiled image (TileWidth/TileLength/TileOffsets/TileByteCounts) of T x T tiles, edge tiles
zero-padded, raw or one zlib stream per tile (`tiff_deflate`).  The reference's TiffWriter
writes one strip (TileRequestHandler.java:176-199); this is an opt-in layout for viewers
that fetch whole-slide TIFFs, so its oracle is our C writer/decoder (oracle/pbx_oracle.c
`pbxo_tiff_tiled_write`, `tiff_decode_tiles`) pinned against tifffile 2021.7.2 (the
image's /opt/conda Python), an independent TIFF reader.

CPU: oracle writer -> oracle decoder and -> tifffile round trips over ragged sizes.
GPU: uncompressed responses equal the oracle writer's bytes exactly; deflate responses
decode (oracle and zlib) to the exact tile, with every TileOffsets / TileByteCounts entry
checked against the zlib stream it points at.
"""
import itertools
import os
import subprocess
import tempfile
import zlib

import pytest

import pbx

CONDA_PY = "/opt/conda/bin/python3.9"
_ids = itertools.count(9000)

# (w, h, T): exact multiples, ragged edges, one tile smaller than T, single column/row
CASES = [(256, 256, 256), (300, 200, 64), (17, 5, 16), (1, 1, 16), (513, 64, 128),
         (64, 700, 256), (1000, 333, 512)]


def _tags(body):
    """IFD entries of a big-endian TIFF: {tag: (type, count, value_or_offset)}."""
    assert body[:4] == b"MM\x00\x2a"
    ifd = int.from_bytes(body[4:8], "big")
    n = int.from_bytes(body[ifd:ifd + 2], "big")
    out = {}
    for k in range(n):
        e = body[ifd + 2 + 12 * k: ifd + 14 + 12 * k]
        typ, cnt = int.from_bytes(e[2:4], "big"), int.from_bytes(e[4:8], "big")
        v = int.from_bytes(e[8:10], "big") if typ == 3 and cnt == 1 else int.from_bytes(e[8:12], "big")
        out[int.from_bytes(e[0:2], "big")] = (typ, cnt, v)
    return out


def _tile_table(body):
    t = _tags(body)
    n = t[324][1]
    if n == 1:
        return [t[324][2]], [t[325][2]]
    o, c = t[324][2], t[325][2]
    offs = [int.from_bytes(body[o + 4 * k: o + 4 * k + 4], "big") for k in range(n)]
    cnts = [int.from_bytes(body[c + 4 * k: c + 4 * k + 4], "big") for k in range(n)]
    return offs, cnts


def _tifffile_decode(blobs):
    """Decode TIFF blobs with tifffile in the conda interpreter; returns big-endian bytes."""
    with tempfile.TemporaryDirectory() as d:
        paths = []
        for i, b in enumerate(blobs):
            p = os.path.join(d, f"{i}.tif")
            with open(p, "wb") as f:
                f.write(b)
            paths.append(p)
        script = ("import sys, tifffile\n"
                  "for p in sys.argv[1:]:\n"
                  "    a = tifffile.imread(p)\n"
                  "    open(p + '.raw', 'wb').write(a.astype(a.dtype.newbyteorder('>')).tobytes())\n")
        subprocess.run([CONDA_PY, "-c", script] + paths, check=True, timeout=120)
        return [open(p + ".raw", "rb").read() for p in paths]


# ------------------------------------------------------------------------------ CPU

@pytest.mark.parametrize("comp", [1, 8])
def test_oracle_tiled_roundtrip(oracle, comp):
    for (w, h, t), pt in itertools.product(CASES, [pbx.UINT8, pbx.UINT16, pbx.FLOAT, pbx.DOUBLE]):
        tile = oracle.gen_region(2, pt, 3, 1, w, h).tobytes()
        bpp = oracle.BPP[pt]
        body = oracle.tiff_tiled_write(tile, w, h, bpp, 1, t, comp)
        r, px, meta = oracle.tiff_decode(body, len(tile))
        assert r == 0 and meta["compression"] == comp and (meta["w"], meta["h"]) == (w, h)
        assert px == tile, (w, h, t, pt, comp)
        tg = _tags(body)
        assert tg[322][2] == t and tg[323][2] == t
        assert tg[324][1] == -(-w // t) * -(-h // t)


def test_oracle_tiled_rejects(oracle):
    tile = bytes(64 * 64 * 2)
    body = bytearray(oracle.tiff_tiled_write(tile, 64, 64, 2, 1, 16, 1))
    r, _, _ = oracle.tiff_decode(bytes(body[:-1]), len(tile))  # truncated last tile
    assert r != 0
    with pytest.raises(ValueError):
        oracle.tiff_tiled_write(tile, 64, 64, 2, 1, 20, 1)  # not a multiple of 16


@pytest.mark.skipif(not os.path.exists(CONDA_PY), reason="no tifffile interpreter")
def test_oracle_tiled_vs_tifffile(oracle):
    blobs, want = [], []
    for (w, h, t), (pt, comp) in zip(CASES, itertools.cycle([(pbx.UINT16, 1), (pbx.UINT8, 8),
                                                             (pbx.FLOAT, 8), (pbx.INT16, 1)])):
        tile = oracle.gen_region(2, pt, 0, 0, w, h).tobytes()
        sf = 3 if pt == pbx.FLOAT else 2 if pt == pbx.INT16 else 1
        blobs.append(oracle.tiff_tiled_write(tile, w, h, oracle.BPP[pt], sf, t, comp))
        want.append(tile)
    assert _tifffile_decode(blobs) == want


def test_config_rejects_bad_tile():
    """Checked before any device query, so it runs without a GPU."""
    for bad in (8, 20, 4112, -16):
        with pytest.raises(pbx.PbxError):
            pbx.PixelsService(tiff_tile=bad)


# ------------------------------------------------------------------------------ GPU

@pytest.fixture(scope="module", params=[(16, False), (64, True), (256, False), (256, True)],
                ids=lambda p: f"T{p[0]}-{'deflate' if p[1] else 'raw'}")
def tiled(request):
    t, dfl = request.param
    s = pbx.PixelsService(tiff_tile=t, tiff_deflate=dfl)
    yield s, t, dfl
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pt", [pbx.INT8, pbx.UINT16, pbx.INT32, pbx.DOUBLE])
@pytest.mark.parametrize("little_endian", [False, True])
def test_gpu_tiled_tiff(tiled, oracle, pt, little_endian):
    svc, t, dfl = tiled
    sx, sy = 1100, 760
    iid = next(_ids)
    plane_be = oracle.gen_region(2, pt, 0, 0, sx, sy, big_endian=True)
    data = oracle.gen_region(2, pt, 0, 0, sx, sy, big_endian=False) if little_endian else plane_be
    svc.register_plane(iid, 0, 0, 0, pt, sx, sy, data=data, big_endian=not little_endian)
    regions = [(0, 0, 256, 256), (3, 5, 300, 200), (1099, 759, 1, 1), (8, 16, 17, 5),
               (0, 0, 0, 0), (64, 128, 513, 64), (1, 2, 64, 700)]
    res = svc.get_tiles([pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format="tif")
                         for (x, y, w, h) in regions])
    bpp = oracle.BPP[pt]
    sf = 3 if pt == pbx.DOUBLE else 2 if pt in (pbx.INT8, pbx.INT32) else 1
    for (x, y, w, h), (st, body) in zip(regions, res):
        w, h = w or sx, h or sy
        assert st == pbx.OK
        tile = oracle.extract_be(plane_be, True, pt, sx * bpp, x, y, w, h).tobytes()
        if not dfl:
            assert body == oracle.tiff_tiled_write(tile, w, h, bpp, sf, t, 1), (t, x, y, w, h)
            continue
        r, px, meta = oracle.tiff_decode(body, len(tile))
        assert r == 0 and meta["compression"] == 8 and px == tile, (t, x, y, w, h)
        offs, cnts = _tile_table(body)
        assert offs[0] == (160 if len(offs) == 1 else (160 + 8 * len(offs) + 15) // 16 * 16)
        for k, (o, c) in enumerate(zip(offs, cnts)):  # every tile is one exact zlib stream
            assert zlib.decompress(body[o:o + c]).__len__() == t * t * bpp
            if k + 1 < len(offs):
                assert o + c == offs[k + 1]
        assert offs[-1] + cnts[-1] == len(body)


@pytest.mark.gpu
def test_gpu_tiled_tiff_mixed_batch(oracle):
    """Tiled-TIFF sub-tiles next to PNG, raw and strip-less batches in one launch: the
    deflate arena keeps each response contiguous."""
    with pbx.PixelsService(tiff_tile=128, tiff_deflate=True) as svc:
        iid = next(_ids)
        sx, sy = 900, 600
        plane = oracle.gen_region(1, pbx.UINT16, 0, 0, sx, sy, big_endian=True)
        svc.register_plane(iid, 0, 0, 0, pbx.UINT16, sx, sy, data=plane, big_endian=True)
        regs = [((37 * i) % 600, (53 * i) % 400, 200 + i, 150 + 2 * i, ("tif", "png", None)[i % 3])
                for i in range(24)]
        res = svc.get_tiles([pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format=f) for x, y, w, h, f in regs])
        for (x, y, w, h, f), (st, body) in zip(regs, res):
            assert st == pbx.OK
            tile = oracle.extract_be(plane, True, pbx.UINT16, sx * 2, x, y, w, h).tobytes()
            if f == "tif":
                r, px, _ = oracle.tiff_decode(body, len(tile))
                assert r == 0 and px == tile
            elif f == "png":
                r, px, _ = oracle.png_decode(body)
                assert r == 0 and px == tile
            else:
                assert body == tile
