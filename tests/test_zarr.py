"""NGFF / Zarr v2 chunk decode into HBM (pbx_plane_register_zarr).

CPU (not gpu): the oracle's frame/codec restatement (oracle/zarr_oracle.c) against the
c-blosc 1.21 / zlib fixtures in tests/golden/zarr (made by imagecodecs, script committed),
and the test-side frame writer (tests/_zarr.py) byte-identical to c-blosc's frames.
GPU: every fixture decoded on the GPU equals the fixture's raw bytes; multi-chunk planes
(edge chunks, missing chunks with fill values, every codec) equal the oracle's assembly of
the same chunks byte for byte; tiles served from a Zarr plane equal the oracle's tiles;
malformed or unsupported chunks fail with 400 and register nothing.
"""
import ctypes
import itertools
import json
import os
import zlib

import numpy as np
import pytest

import _zarr

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "zarr")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))
CASES = MANIFEST["cases"]
CODEC = {"blosc": 1, "zlib": 2, None: 0}
PT = {"i1": 0, "u1": 1, "i2": 2, "u2": 3, "i4": 4, "u4": 5, "f4": 6, "f8": 7}

_ids = itertools.count(900000)  # disjoint from the other test files (shared service)


def fixture(name):
    enc = open(os.path.join(GOLD, name + ".enc"), "rb").read()
    raw = open(os.path.join(GOLD, name + ".raw"), "rb").read()
    return enc, raw


def oracle_decode(oracle, codec, enc, nbytes):
    L = oracle.lib()
    out = ctypes.create_string_buffer(max(nbytes, 1))
    rc = L.pbxo_zarr_decode_chunk(CODEC[codec], enc, ctypes.c_size_t(len(enc)), out,
                                  ctypes.c_size_t(nbytes))
    return rc, out.raw[:nbytes]


def oracle_plane(oracle, codec, bpp, sx, sy, cx, cy, chunks, fill_bytes):
    L = oracle.lib()
    lens = [len(c) if c else 0 for c in chunks]
    offs = (ctypes.c_uint64 * (len(chunks) + 1))(*np.concatenate([[0], np.cumsum(lens)]).astype(int).tolist())
    data = b"".join(c for c in chunks if c) or b"\0"
    out = ctypes.create_string_buffer(sx * sy * bpp)
    rc = L.pbxo_zarr_plane(CODEC[codec], bpp, sx, sy, cx, cy, data, offs, fill_bytes, out)
    assert rc == 0
    return out.raw


# ----------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_decodes_fixture(oracle, case):
    enc, raw = fixture(case["name"])
    rc, out = oracle_decode(oracle, case["codec"], enc, len(raw))
    assert rc == 0 and out == raw


CB_CASES = [(cn, sh, dt) for cn in ("blosclz", "lz4", "lz4hc", "zlib", "zstd") for sh in (0, 1, 2)
            for dt in (">u2", "u1", "<f4", ">f8")]


@pytest.mark.parametrize("cname,shuffle,dtype", CB_CASES)
def test_oracle_matches_cblosc(oracle, cname, shuffle, dtype):
    """The oracle's c-blosc frame restatement (blosclz, bit shuffle, zstd via the system
    libzstd) decodes frames the real c-blosc 1.21 wrote exactly as c-blosc itself does, for
    odd sizes (leftover blocks, element counts not a multiple of 8) and explicit block sizes."""
    if _zarr.cblosc() is None:
        pytest.skip("c-blosc 1.21 library not in this image")
    for h, w, bs in ((61, 67, 0), (256, 200, 0), (128, 130, 4096), (97, 101, 24576)):
        plane = _zarr.noise_plane(h, w, dtype, seed=h + w)
        raw = plane.tobytes()
        enc = _zarr.cblosc_encode(raw, plane.dtype.itemsize, cname, 5, shuffle, bs)
        rc, out = oracle_decode(oracle, "blosc", enc, len(raw))
        assert rc == 0 and out == raw == _zarr.cblosc_decode(enc, len(raw)), (h, w, bs)


@pytest.mark.parametrize("case", [c for c in CASES if c["codec"] == "blosc"
                                  and c["params"]["compressor"] in ("lz4", "zlib")
                                  and c["params"]["shuffle"] in (0, 1)],
                         ids=lambda c: c["name"])
def test_frame_writer_matches_cblosc(case):
    enc, raw = fixture(case["name"])
    p = case["params"]
    mine = _zarr.blosc_encode(raw, np.dtype(case["dtype"]).itemsize, clevel=p["level"],
                              shuffle=bool(p["shuffle"]), codec=p["compressor"])
    assert mine == enc


def test_oracle_plane_assembly(oracle):
    plane = _zarr.noise_plane(300, 200, ">u2", seed=3)
    chunks = _zarr.encode_chunks(plane, 64, 48, "blosc")
    chunks[5] = None
    got = np.frombuffer(oracle_plane(oracle, "blosc", 2, 200, 300, 48, 64, chunks,
                                     (7).to_bytes(2, "big")), ">u2").reshape(300, 200)
    want = plane.copy()
    gx = -(-200 // 48)
    cy, cx = divmod(5, gx)
    want[cy * 64:(cy + 1) * 64, cx * 48:(cx + 1) * 48] = 7
    assert np.array_equal(got, want)


def _write_ngff(root, shape, chunks, dtype, sep, compressor, fill=0, skip=()):
    """A Zarr v2 array directory; returns {lead index tuple: plane array}."""
    root.mkdir(parents=True, exist_ok=True)
    meta = {"zarr_format": 2, "shape": list(shape), "chunks": list(chunks), "dtype": dtype,
            "order": "C", "fill_value": fill, "filters": None, "dimension_separator": sep,
            "compressor": None if compressor is None else {"id": compressor}}
    (root / ".zarray").write_text(json.dumps(meta))
    planes = {}
    for lead in np.ndindex(*shape[:-2]):
        p = _zarr.noise_plane(shape[-2], shape[-1], dtype, seed=sum(lead) + 7)
        planes[lead] = p
        gx = -(-shape[-1] // chunks[-1])
        for k, ch in enumerate(_zarr.encode_chunks(p, chunks[-2], chunks[-1], compressor)):
            j, i = divmod(k, gx)
            if (lead, j, i) in skip:
                continue
            path = root / sep.join(str(v) for v in list(lead) + [j, i])
            path.parent.mkdir(parents=True, exist_ok=True)
            path.write_bytes(ch)
    return planes


@pytest.mark.parametrize("ndim,sep", [(5, "/"), (3, "."), (2, ".")])
def test_ngff_plane_spec(tmp_path, ndim, sep):
    """NGFF array reading on the host (which chunk files belong to a plane, dtype, fill)."""
    import pbx
    shape = [2, 3, 4, 70, 90][5 - ndim:]
    chunks = [1] * (ndim - 2) + [32, 40]
    lead0 = tuple([1, 2, 3][3 - (ndim - 2):]) if ndim > 2 else ()
    planes = _write_ngff(tmp_path / "a", shape, chunks, "<u2", sep, "zlib", fill=9,
                         skip={(lead0, 1, 2)})
    z, c, t = (3 if ndim >= 3 else 0), (2 if ndim >= 4 else 0), (1 if ndim >= 5 else 0)
    sp = pbx.zarr_plane_spec(str(tmp_path / "a"), 77, z, c, t)
    assert (sp["size_x"], sp["size_y"], sp["chunk_x"], sp["chunk_y"]) == (90, 70, 40, 32)
    assert sp["pixel_type"] == pbx.UINT16 and sp["big_endian"] is False and sp["fill_bits"] == 9
    assert sp["codec"] == "zlib" and len(sp["chunks"]) == 3 * 3
    assert sp["chunks"][1 * 3 + 2] is None  # the skipped chunk file
    dec = zlib.decompress(sp["chunks"][0])
    assert dec == _zarr.chunk_grid(planes[lead0], 32, 40)[0].tobytes()
    with pytest.raises(pbx.PbxError):
        pbx.zarr_plane_spec(str(tmp_path / "a"), 77, 99 if ndim >= 3 else 0, c, t + (ndim < 3))


# ----------------------------------------------------------------------------- GPU
gpu = pytest.mark.gpu


def plane_be(service, pid, dtype, h, w):
    raw = service.read_plane_be(pid, h * w * np.dtype(dtype).itemsize)
    return np.frombuffer(raw, np.dtype(dtype).newbyteorder(">")).reshape(h, w)


@gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_decodes_fixture(service, case):
    import pbx
    enc, raw = fixture(case["name"])
    h, w = case["shape"]
    dt = np.dtype(case["dtype"])
    iid = next(_ids)
    args = (iid, 0, 0, 0, PT[dt.str[1:]], w, h, w, h, case["codec"], [enc])
    pid = service.register_zarr_plane(*args, big_endian=dt.str[0] != "<")
    got = plane_be(service, pid, dt, h, w)
    want = np.frombuffer(raw, dt).reshape(h, w)
    assert np.array_equal(got.view(np.uint8), want.astype(dt.newbyteorder(">")).view(np.uint8))
    service.release_plane(pid)


@gpu
@pytest.mark.parametrize("codec,kw", [
    ("blosc", dict(codec="lz4", clevel=5)),
    ("blosc", dict(codec="lz4", clevel=9, shuffle=False)),
    ("blosc", dict(codec="lz4", clevel=1, blocksize=4096)),
    ("blosc", dict(codec="zlib", clevel=5)),
    ("blosc", dict(codec="lz4", clevel=5, split=False)),
    ("zlib", dict(level=1)),
    ("zlib", dict(level=6)),
    ("zlib", dict(level=9)),
    (None, {}),
], ids=["lz4", "lz4-noshuffle-l9", "lz4-4k-blocks", "blosc-zlib", "lz4-nosplit", "zlib1", "zlib6",
        "zlib9", "raw"])
@pytest.mark.parametrize("dtype", [">u2", "<u2", "u1", ">f4", "<i4", ">f8"])
def test_gpu_plane_multichunk(service, oracle, codec, kw, dtype):
    h, w, cy, cx = 333, 517, 96, 128  # edge chunks in both directions
    dt = np.dtype(dtype)
    plane = _zarr.noise_plane(h, w, dtype, seed=len(dtype) + h)
    if dt.kind == "f":
        plane = (plane.astype(np.float64) * 0.25).astype(dtype)
    chunks = _zarr.encode_chunks(plane, cy, cx, codec, **kw)
    chunks[1] = None       # missing chunks read as fill_value
    chunks[-1] = b""
    fill_val = np.array([3], dtype=dt.newbyteorder("="))
    fill_bits = int(fill_val.view("u%d" % dt.itemsize)[0])
    iid = next(_ids)
    pid, (ms_dec, ms_place) = service.register_zarr_plane(
        iid, 0, 0, 0, PT[dt.str[1:]], w, h, cx, cy, codec, chunks,
        big_endian=dt.str[0] != "<", fill_bits=fill_bits, timing=True)
    assert ms_dec >= 0 and ms_place >= 0
    want = oracle_plane(oracle, codec, dt.itemsize, w, h, cx, cy, chunks,
                        fill_val.astype(dt).tobytes())
    want = np.frombuffer(want, dt).reshape(h, w)
    got = plane_be(service, pid, dt, h, w)
    assert np.array_equal(got.view(np.uint8), want.astype(dt.newbyteorder(">")).view(np.uint8))
    service.release_plane(pid)


@gpu
def test_gpu_zarr_tiles_png_raw_tif(service, oracle):
    """Tiles served from a Zarr-decoded plane equal the oracle's tiles of the same pixels."""
    import pbx
    h, w = 1024, 1536
    plane = _zarr.noise_plane(h, w, ">u2", seed=11)
    chunks = _zarr.encode_chunks(plane, 512, 512, "blosc")
    iid = next(_ids)
    pid = service.register_zarr_plane(iid, 0, 0, 0, pbx.UINT16, w, h, 512, 512, "blosc", chunks)
    be = plane.tobytes()
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, 256, 256, 512, 512, format="png"),
            pbx.TileCtx(iid, 0, 0, 0, 1000, 700, 536, 324),
            pbx.TileCtx(iid, 0, 0, 0, 0, 0, 300, 200, format="tif")]
    (s1, png), (s2, raw), (s3, tif) = service.get_tiles(ctxs)
    assert (s1, s2, s3) == (0, 0, 0)
    r, px, _ = oracle.png_decode(png)
    assert r == 0 and px == oracle.extract_be(np.frombuffer(be, np.uint8), True, pbx.UINT16, w * 2,
                                              256, 256, 512, 512).tobytes()
    assert raw == oracle.extract_be(np.frombuffer(be, np.uint8), True, pbx.UINT16, w * 2,
                                    1000, 700, 536, 324).tobytes()
    r, px, _ = oracle.tiff_decode(tif, 300 * 200 * 2)
    assert r == 0 and px == oracle.extract_be(np.frombuffer(be, np.uint8), True, pbx.UINT16, w * 2,
                                              0, 0, 300, 200).tobytes()
    service.release_plane(pid)


@gpu
def test_gpu_ngff_directory(service, oracle, tmp_path):
    """register_zarr_array reads an NGFF (t, c, z, y, x) array directory like JZarr does."""
    import pbx
    t_, c_, z_, h, w = 1, 2, 3, 400, 600
    arr = tmp_path / "0"
    arr.mkdir()
    meta = {"zarr_format": 2, "shape": [t_, c_, z_, h, w], "chunks": [1, 1, 1, 256, 256],
            "dtype": ">u2", "order": "C", "fill_value": 0, "filters": None,
            "dimension_separator": "/",
            "compressor": {"id": "blosc", "cname": "lz4", "clevel": 5, "shuffle": 1, "blocksize": 0}}
    (arr / ".zarray").write_text(json.dumps(meta))
    planes = {}
    for c in range(c_):
        for z in range(z_):
            p = _zarr.noise_plane(h, w, ">u2", seed=10 * c + z)
            planes[(c, z)] = p
            for k, ch in enumerate(_zarr.encode_chunks(p, 256, 256, "blosc")):
                j, i = divmod(k, 3)
                d = arr / "0" / str(c) / str(z) / str(j)
                d.mkdir(parents=True, exist_ok=True)
                (d / str(i)).write_bytes(ch)
    iid = next(_ids)
    pid = service.register_zarr_array(str(arr), iid, 2, 1, 0)
    got = plane_be(service, pid, ">u2", h, w)
    assert np.array_equal(got, planes[(1, 2)])
    st, raw = service.get_tile(pbx.TileCtx(iid, 2, 1, 0, 100, 50, 64, 32))
    assert st == 0 and raw == planes[(1, 2)][50:82, 100:164].tobytes()
    service.release_plane(pid)


@gpu
@pytest.mark.parametrize("damage", ["truncate", "flip", "bad_offset"])
def test_gpu_corrupt_chunk_is_400(service, damage):
    import pbx
    plane = _zarr.noise_plane(256, 256, ">u2", seed=1)
    chunks = _zarr.encode_chunks(plane, 128, 128, "blosc")
    c = bytearray(chunks[2])
    if damage == "truncate":
        c = c[:len(c) // 2]
    elif damage == "flip":
        # corrupt LZ4 sequences inside the first split (after header, block table, csize)
        for k in range(40, min(len(c), 400), 7):
            c[k] ^= 0xA5
    else:
        c[16:20] = (len(c) + 100).to_bytes(4, "little")
    chunks[2] = bytes(c)
    iid = next(_ids)
    with pytest.raises(pbx.PbxError) as ei:
        service.register_zarr_plane(iid, 0, 0, 0, pbx.UINT16, 256, 256, 128, 128, "blosc", chunks)
    assert ei.value.status == 400
    # nothing registered: the same key registers cleanly afterwards
    good = _zarr.encode_chunks(plane, 128, 128, "blosc")
    pid = service.register_zarr_plane(iid, 0, 0, 0, pbx.UINT16, 256, 256, 128, 128, "blosc", good)
    assert np.array_equal(plane_be(service, pid, ">u2", 256, 256), plane)
    service.release_plane(pid)


@gpu
def test_gpu_corrupt_zlib_is_400(service):
    import pbx
    plane = _zarr.noise_plane(128, 128, ">u2", seed=2)
    enc = bytearray(zlib.compress(plane.tobytes(), 6))
    for k in range(20, 200, 5):
        enc[k] ^= 0x3C
    with pytest.raises(pbx.PbxError) as ei:
        service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, 128, 128, 128, 128, "zlib",
                                    [bytes(enc)])
    assert ei.value.status == 400


@gpu
@pytest.mark.parametrize("compressor,kw", [("blosc", {}), ("zlib", {"level": 1}), ("blosc", {"codec": "zlib"})],
                         ids=["blosc-lz4", "zlib1", "blosc-zlib"])
def test_gpu_zarr_full_size(service, compressor, kw):
    """A 8192^2 uint16 plane of 512^2 chunks (256 chunks; blosc: 1,024 streams)."""
    import pbx
    h = w = 8192
    plane = _zarr.noise_plane(h, w, ">u2", seed=5)
    chunks = _zarr.encode_chunks(plane, 512, 512, compressor, **kw)
    pid, (ms_dec, ms_place) = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, w, h,
                                                          512, 512, compressor, chunks, timing=True)
    assert np.array_equal(plane_be(service, pid, ">u2", h, w), plane)
    print("%s: decode %.3f ms, place %.3f ms" % (compressor, ms_dec, ms_place))
    service.release_plane(pid)


@gpu
def test_gpu_planes_one_launch(service, oracle):
    """Several planes (mixed codecs and dtypes) decoded by one pbx_planes_register_zarr call;
    a corrupt chunk in any of them registers none."""
    import pbx
    specs, wants = [], []
    for k, (comp, kw, dtype, cy, cx) in enumerate([("blosc", {}, ">u2", 128, 128),
                                                    ("zlib", {"level": 6}, "<u2", 96, 200),
                                                    ("blosc", {"codec": "zlib"}, ">f4", 64, 64),
                                                    (None, {}, "u1", 100, 100)]):
        dt = np.dtype(dtype)
        plane = _zarr.noise_plane(300, 260, dtype, seed=40 + k)
        chunks = _zarr.encode_chunks(plane, cy, cx, comp, **kw)
        chunks[0] = None
        iid = next(_ids)
        specs.append(dict(image_id=iid, z=k, c=0, t=0, pixel_type=PT[dt.str[1:]], size_x=260,
                          size_y=300, chunk_x=cx, chunk_y=cy, codec=comp, chunks=chunks,
                          big_endian=dt.str[0] != "<", fill_bits=0))
        want = plane.copy()
        want[:cy, :cx] = 0
        wants.append(want)
    bad = [dict(sp) for sp in specs]
    ch = list(bad[1]["chunks"])
    ch[3] = ch[3][:len(ch[3]) // 3]
    bad[1]["chunks"] = ch
    with pytest.raises(pbx.PbxError) as ei:
        service.register_zarr_planes(bad)
    assert ei.value.status == 400
    clash = [dict(specs[0]), dict(specs[0], z=9, size_x=259)]  # same image, other size
    with pytest.raises(pbx.PbxError) as ei:
        service.register_zarr_planes(clash)
    assert ei.value.status == 400
    ids, (ms_dec, ms_place) = service.register_zarr_planes(specs, timing=True)
    assert len(ids) == 4 and ms_dec > 0
    for pid, sp, want in zip(ids, specs, wants):
        dt = want.dtype
        got = plane_be(service, pid, dt, 300, 260)
        assert np.array_equal(got.view(np.uint8), want.astype(dt.newbyteorder(">")).view(np.uint8))
        service.release_plane(pid)


@gpu
def test_gpu_ngff_all_planes_one_call(service, tmp_path):
    """register_zarr_array_planes: every (z, c, t) plane of an NGFF array in one launch."""
    import pbx
    planes = _write_ngff(tmp_path / "img", [2, 2, 3, 200, 300], [1, 1, 1, 128, 128], ">u2", "/",
                         "blosc")
    iid = next(_ids)
    ids = service.register_zarr_array_planes(str(tmp_path / "img"), iid)
    assert len(ids) == 12
    for (z, c, t), pid in ids.items():
        assert np.array_equal(plane_be(service, pid, ">u2", 200, 300), planes[(t, c, z)])
    st, raw = service.get_tile(pbx.TileCtx(iid, 2, 1, 1, 10, 20, 30, 40))
    assert st == 0 and raw == planes[(1, 1, 2)][20:60, 10:40].tobytes()
    for pid in ids.values():
        service.release_plane(pid)


def _flushed_zlib(raw, level, piece_sizes):
    """A zlib stream whose pieces are separated by Z_SYNC_FLUSH (each flush ends with an
    empty stored block: LEN 0 after byte alignment), or at level 0 stored blocks of 1..3
    bytes: blocks shorter than the bytes the decoder's bit buffer holds."""
    co = zlib.compressobj(level)
    out, pos, k = [], 0, 0
    while pos < len(raw):
        n = piece_sizes[k % len(piece_sizes)]
        out.append(co.compress(raw[pos:pos + n]))
        out.append(co.flush(zlib.Z_SYNC_FLUSH))
        pos += n
        k += 1
    out.append(co.flush())
    return b"".join(out)


@gpu
@pytest.mark.parametrize("level,pieces", [(6, [777, 1, 4096, 3]), (0, [1, 2, 3]), (1, [2, 5000]),
                                          (0, [65535, 1])],
                         ids=["l6-sync", "l0-tiny-stored", "l1-sync", "l0-max-stored"])
def test_gpu_inflate_sync_flush_and_tiny_stored_blocks(service, oracle, level, pieces):
    """Stored blocks of 0..3 bytes (sync flushes; level 0 pieces) decode exactly like zlib's
    inflate (the oracle's uncompress): the bytes buffered past such a block are not lost."""
    import pbx
    h, w = 64, 96
    plane = _zarr.noise_plane(h, w, ">u2", seed=17)
    raw = plane.tobytes()
    enc = _flushed_zlib(raw, level, pieces)
    assert zlib.decompress(enc) == raw
    rc, want = oracle_decode(oracle, "zlib", enc, len(raw))
    assert rc == 0 and want == raw
    pid = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, w, h, w, h, "zlib", [enc])
    assert np.array_equal(plane_be(service, pid, ">u2", h, w), plane)
    service.release_plane(pid)


def _strategy_plane(kind, h, w):
    """Planes whose deflate streams stress different paths of the self-synchronizing decoder:
    long runs (258-byte matches at distance 1-2), short codes (many tokens per segment: the
    FIFO-room truncation of a macro-round), smooth data, and noise."""
    rng = np.random.default_rng(23)
    if kind == "zeros":
        return np.zeros((h, w), ">u2")
    if kind == "steps":
        return (np.arange(h * w, dtype=np.uint32) // 1000 % 7).astype(">u2").reshape(h, w)
    if kind == "gradient":
        return (np.add.outer(np.arange(h), np.arange(w)) * 13).astype(">u2")
    if kind == "sparse":
        p = np.zeros((h, w), ">u2")
        p.flat[rng.integers(0, h * w, h * w // 50)] = rng.integers(0, 65535, h * w // 50)
        return p
    return rng.integers(0, 4096, (h, w)).astype(">u2")


@gpu
@pytest.mark.parametrize("strategy", [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE,
                                      zlib.Z_FIXED], ids=["default", "filtered", "huffman-only", "rle", "fixed"])
@pytest.mark.parametrize("kind", ["zeros", "steps", "gradient", "sparse", "noise12"])
@pytest.mark.parametrize("level", [1, 9])
def test_gpu_inflate_strategies(service, oracle, strategy, kind, level):
    """zlib streams of every deflate strategy (fixed and dynamic codes, literal-only, run-length
    only) over compressible and noisy planes decode exactly like zlib's inflate."""
    import pbx
    h, w = 300, 520
    plane = _strategy_plane(kind, h, w)
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 9, strategy)
    enc = co.compress(plane.tobytes()) + co.flush()
    pid = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, w, h, w, h, "zlib", [enc])
    assert np.array_equal(plane_be(service, pid, ">u2", h, w), plane)
    service.release_plane(pid)


@gpu
@pytest.mark.parametrize("cname", ["blosclz", "zstd", "lz4", "zlib"])
@pytest.mark.parametrize("shuffle", [0, 1, 2], ids=["noshuffle", "shuffle", "bitshuffle"])
@pytest.mark.parametrize("dtype", [">u2", "u1", "<i4", ">f8"])
def test_gpu_cblosc_codecs(service, oracle, cname, shuffle, dtype):
    """Chunks written by the real c-blosc 1.21 with every codec the NGFF writers use and
    every shuffle mode, multi-chunk planes with edge and missing chunks: the GPU plane equals
    the oracle's assembly (and c-blosc's own decode) byte for byte."""
    if _zarr.cblosc() is None:
        pytest.skip("c-blosc 1.21 library not in this image")
    h, w, cy, cx = 301, 257, 128, 96
    dt = np.dtype(dtype)
    plane = _zarr.noise_plane(h, w, dtype, seed=len(cname) + shuffle)
    chunks = _zarr.encode_chunks(plane, cy, cx, "blosc", cname=cname, clevel=5, shuffle=shuffle)
    chunks[2] = None
    for c, raw in zip(chunks, _zarr.chunk_grid(plane, cy, cx)):
        if c:
            assert _zarr.cblosc_decode(c, raw.nbytes) == raw.tobytes()
    iid = next(_ids)
    pid = service.register_zarr_plane(iid, 0, 0, 0, PT[dt.str[1:]], w, h, cx, cy, "blosc", chunks,
                                      big_endian=dt.str[0] != "<", fill_bits=0)
    want = oracle_plane(oracle, "blosc", dt.itemsize, w, h, cx, cy, chunks, bytes(dt.itemsize))
    want = np.frombuffer(want, dt).reshape(h, w)
    got = plane_be(service, pid, dt, h, w)
    assert np.array_equal(got.view(np.uint8), want.astype(dt.newbyteorder(">")).view(np.uint8))
    service.release_plane(pid)


@gpu
@pytest.mark.parametrize("cname,clevel", [("zstd", 1), ("zstd", 9), ("blosclz", 9), ("zstd", 5)])
def test_gpu_cblosc_full_size(service, cname, clevel):
    """A 4096^2 uint16 plane of 512^2 c-blosc chunks (256 chunks), G_NOISE-like and smooth
    halves, decoded exactly."""
    if _zarr.cblosc() is None:
        pytest.skip("c-blosc 1.21 library not in this image")
    import pbx
    h = w = 4096
    plane = _zarr.noise_plane(h, w, ">u2", seed=clevel)
    plane[:, w // 2:] = (np.arange(w // 2)[None, :] // 7 + np.arange(h)[:, None] // 5).astype(">u2")
    chunks = _zarr.encode_chunks(plane, 512, 512, "blosc", cname=cname, clevel=clevel, shuffle=1)
    pid, (ms_dec, ms_place) = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, w, h, 512,
                                                          512, "blosc", chunks, timing=True)
    assert np.array_equal(plane_be(service, pid, ">u2", h, w), plane)
    print("%s-%d: decode %.3f ms, place %.3f ms" % (cname, clevel, ms_dec, ms_place))
    service.release_plane(pid)


@gpu
@pytest.mark.parametrize("damage", ["snappy", "version3", "zstd_flip", "blosclz_trunc"])
def test_gpu_cblosc_rejects(service, damage):
    """Frames the decoders cannot or must not take fail the plane with 400: snappy (codec 2),
    a blosc2-era format version, corrupt zstd and truncated blosclz streams."""
    if _zarr.cblosc() is None:
        pytest.skip("c-blosc 1.21 library not in this image")
    import pbx
    plane = _zarr.noise_plane(128, 128, ">u2", seed=4)
    cname = "zstd" if damage.startswith("zstd") else "blosclz" if damage.startswith("blosclz") else "lz4"
    enc = bytearray(_zarr.cblosc_encode(plane.tobytes(), 2, cname, 5, 1))
    if damage == "snappy":
        enc[2] = (enc[2] & 0x1F) | (2 << 5)
    elif damage == "version3":
        enc[0] = 3
    elif damage == "zstd_flip":
        for k in range(40, len(enc) - 8, 11):
            enc[k] ^= 0x5A
    else:
        enc[12:16] = (len(enc) - 40).to_bytes(4, "little")
        enc = enc[:len(enc) - 40]
    with pytest.raises(pbx.PbxError) as ei:
        service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, 128, 128, 128, 128, "blosc",
                                    [bytes(enc)])
    assert ei.value.status == 400


def _write_ngff_image(root, levels, dtype=">u2", axes=("t", "c", "z", "y", "x"), lead=(1, 2, 3),
                      h=600, w=500, chunk=(128, 96), compressor="blosc", b2r=False):
    """An NGFF multiscale image: dataset k = 2^k-downsampled planes (numpy box means of the
    level above, as a writer would produce), .zattrs multiscales with the given axes; with
    b2r, inside a bioformats2raw container (root/.zattrs layout 3, series 0)."""
    import pathlib
    root = pathlib.Path(root)
    img = root / "0" if b2r else root
    img.mkdir(parents=True, exist_ok=True)
    if b2r:
        (root / ".zattrs").write_text(json.dumps({"bioformats2raw.layout": 3}))
    datasets, arrays = [], []
    for k in range(levels):
        hk, wk = -(-h // 2 ** k), -(-w // 2 ** k)
        shape = list(lead) + [hk, wk]
        planes = _write_ngff(img / str(k), shape, [1] * len(lead) + list(chunk), dtype, "/", compressor)
        arrays.append(planes)
        datasets.append({"path": str(k), "coordinateTransformations": [{"type": "scale", "scale": [1.0] * len(lead) + [2.0 ** k] * 2}]})
    ms = {"multiscales": [{"version": "0.4", "name": "img", "axes": [{"name": a} for a in axes],
                           "datasets": datasets}]}
    (img / ".zattrs").write_text(json.dumps(ms))
    return arrays


@pytest.mark.parametrize("axes,lead", [(("t", "c", "z", "y", "x"), (1, 2, 3)), (("c", "y", "x"), (2,)),
                                       (("z", "y", "x"), (3,))])
def test_ngff_axes_planes(tmp_path, axes, lead):
    """Plane enumeration and chunk paths follow the multiscales "axes" (CPU)."""
    import pbx
    _write_ngff_image(tmp_path / "img", 2, axes=axes, lead=lead, h=70, w=50, chunk=(32, 32))
    ms, root = pbx.ngff_multiscales(str(tmp_path / "img"))
    meta = pbx.zarr_array_meta(os.path.join(root, "1"))
    planes = pbx.PixelsService._array_planes(meta, ms["axes"])
    n = int(np.prod(lead))
    assert len(planes) == n
    for z, c, t in planes:
        sp = pbx.zarr_plane_spec(os.path.join(root, "1"), 1, z, c, t, 1, meta, ms["axes"])
        assert sp["level"] == 1 and (sp["size_y"], sp["size_x"]) == (35, 25)
        assert all(ch is not None for ch in sp["chunks"])


@gpu
@pytest.mark.parametrize("b2r", [False, True], ids=["ngff", "bioformats2raw"])
def test_gpu_ngff_pyramid_one_call(service, tmp_path, b2r):
    """A whole 3-level NGFF image (2 channels x 3 z) registers with ONE call; tiles follow
    OMERO's resolution numbering (resolution 2 = dataset 0 = full resolution, 0 = the
    smallest), absent resolution = full resolution, w/h defaults to the full-resolution size."""
    import pbx
    arrays = _write_ngff_image(tmp_path / "img", 3, b2r=b2r)
    iid = next(_ids)
    reg = service.register_ngff_image(str(tmp_path / "img"), iid)
    assert sorted(reg) == [0, 1, 2] and all(len(v) == 6 for v in reg.values())
    z, c = 2, 1
    ctxs = [pbx.TileCtx(iid, z, c, 0, 100, 50, 64, 32),                   # full resolution
            pbx.TileCtx(iid, z, c, 0, 100, 50, 64, 32, resolution=2),     # = dataset 0
            pbx.TileCtx(iid, z, c, 0, 10, 20, 64, 32, resolution=1),      # dataset 1
            pbx.TileCtx(iid, z, c, 0, 3, 4, 100, 60, resolution=0),       # dataset 2 (150 x 125)
            pbx.TileCtx(iid, z, c, 0, 0, 0, 0, 0, resolution=0),          # w/h 500 x 600 > level
            pbx.TileCtx(iid, z, c, 0, 0, 0, 16, 16, resolution=3)]        # no 4th level
    res = service.get_tiles(ctxs)
    lv = [arrays[k][(0, c, z)] for k in range(3)]
    assert res[0] == (0, lv[0][50:82, 100:164].tobytes()) == res[1]
    assert res[2] == (0, lv[1][20:52, 10:74].tobytes())
    assert res[3] == (0, lv[2][4:64, 3:103].tobytes())
    assert res[4][0] == pbx.E_NOTFOUND and res[5][0] == pbx.E_NOTFOUND
    for lvl in reg.values():
        for pid in lvl.values():
            service.release_plane(pid)


def _corruptions(enc: bytes, seed: int, hdr: int):
    """Deterministic damage to one compressed stream: byte flips after the header, a
    truncation, or a garbage tail."""
    rng = np.random.default_rng(seed)
    b = bytearray(enc)
    kind = seed % 4
    if kind == 0:
        for _ in range(int(rng.integers(1, 5))):
            b[int(rng.integers(hdr, len(b)))] ^= int(rng.integers(1, 256))
    elif kind == 1:
        b = b[:int(rng.integers(hdr, len(b)))]
    elif kind == 2:
        k = int(rng.integers(hdr, len(b)))
        b[k:] = rng.integers(0, 256, len(b) - k, dtype=np.uint8).tobytes()
    else:
        k = int(rng.integers(hdr, len(b) - 8))
        b[k:k + 8] = b"\xff" * 8
    return bytes(b)


@gpu
@pytest.mark.parametrize("codec", ["zlib1", "zlib9-fixed", "zlib6-rle", "blosc-zstd", "blosc-lz4", "blosc-blosclz"])
def test_gpu_corrupt_streams_fuzz(service, codec):
    """Damaged streams of every decoder (flipped bytes, truncation, garbage tails) either fail the
    call with 400 or decode; a stream the CPU codec accepts decodes to the same bytes.  (No
    fault, no hang: every decoder's loops are bounded by the stream and output lengths.)"""
    import pbx
    h, w = 96, 128
    plane = _zarr.noise_plane(h, w, ">u2", seed=41) & 0x0FFF
    raw = plane.tobytes()
    if codec.startswith("zlib"):
        level = int(codec[4])
        strat = zlib.Z_FIXED if codec.endswith("fixed") else zlib.Z_RLE if codec.endswith("rle") else 0
        co = zlib.compressobj(level, zlib.DEFLATED, 15, 9, strat)
        enc, comp, hdr = co.compress(raw) + co.flush(), "zlib", 2
        ref = lambda b: zlib.decompress(b)
    else:
        if _zarr.cblosc() is None:
            pytest.skip("c-blosc not in this image")
        enc, comp, hdr = _zarr.cblosc_encode(raw, 2, codec.split("-")[1], 5, 1), "blosc", 16
        ref = lambda b: _zarr.cblosc_decode(b, len(raw))
    ok = failed = 0
    for seed in range(24):
        bad = _corruptions(enc, seed, hdr)
        try:
            want = ref(bad)
        except Exception:
            want = None
        try:
            pid = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, w, h, w, h, comp, [bad])
        except pbx.PbxError as e:
            assert e.status == 400
            failed += 1
            continue
        got = plane_be(service, pid, ">u2", h, w).tobytes()
        service.release_plane(pid)
        if want is not None and len(want) == len(raw):
            assert got == want, seed
        ok += 1
    assert failed > 0


@gpu
def test_gpu_zlib_adler_mismatch_is_400(service):
    """A zlib stream whose deflate data is intact but whose Adler-32 trailer is wrong fails like
    java.util.zip.Inflater ('incorrect data check'); the intact stream decodes."""
    import pbx
    plane = _zarr.noise_plane(64, 96, ">u2", seed=8)
    enc = bytearray(zlib.compress(plane.tobytes(), 6))
    pid = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, 96, 64, 96, 64, "zlib", [bytes(enc)])
    assert np.array_equal(plane_be(service, pid, ">u2", 64, 96), plane)
    service.release_plane(pid)
    enc[-1] ^= 1
    with pytest.raises(zlib.error):
        zlib.decompress(bytes(enc))
    with pytest.raises(pbx.PbxError) as ei:
        service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, 96, 64, 96, 64, "zlib", [bytes(enc)])
    assert ei.value.status == 400


def _zstd_checksummed_chunk(seed=12):
    """A 96 x 128 uint16 chunk as a blosc frame whose zstd streams carry the optional XXH64
    content checksum (c-blosc writes none; libzstd, the reference path's codec, verifies it),
    and the same chunk with the last checksum byte flipped."""
    plane = (_zarr.noise_plane(96, 128, ">u2", seed=seed) & 0x0FFF).astype(">u2")  # (& gives native order)
    enc = _zarr.blosc_encode(plane.tobytes(), 2, 5, True, "zstd", split=False, zstd_checksum=True)
    assert enc[2] & 0x2 == 0  # compressed, not memcpyed: the last bytes are the checksum
    bad = bytearray(enc)
    bad[-1] ^= 0x40
    return plane, enc, bytes(bad)


def test_oracle_zstd_content_checksum(oracle):
    """The oracle (libzstd) decodes checksummed zstd splits and rejects a wrong checksum."""
    import ctypes
    plane, enc, bad = _zstd_checksummed_chunk()
    out = ctypes.create_string_buffer(plane.nbytes)
    offs = (ctypes.c_uint64 * 2)(0, len(enc))
    assert oracle.lib().pbxo_zarr_plane(1, 2, 128, 96, 128, 96, enc, offs, b"\0\0", out) == 0
    assert out.raw == plane.tobytes()
    offs = (ctypes.c_uint64 * 2)(0, len(bad))
    assert oracle.lib().pbxo_zarr_plane(1, 2, 128, 96, 128, 96, bad, offs, b"\0\0", out) != 0


@gpu
def test_gpu_zstd_content_checksum(service):
    """zstd frames with Content_Checksum_flag: the GPU verifies XXH64 of what it decoded
    (as libzstd does): the intact chunk decodes exactly, a wrong checksum fails with 400."""
    import pbx
    plane, enc, bad = _zstd_checksummed_chunk()
    pid = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, 128, 96, 128, 96, "blosc", [enc])
    assert np.array_equal(plane_be(service, pid, ">u2", 96, 128), plane)
    service.release_plane(pid)
    with pytest.raises(pbx.PbxError) as ei:
        service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, 128, 96, 128, 96, "blosc", [bad])
    assert ei.value.status == 400
    # larger frames (many 32-byte stripes, a tail) through the same check
    big = _zarr.noise_plane(512, 512, ">u2", seed=3)
    chunks = [_zarr.blosc_encode(c.tobytes(), 2, 3, True, "zstd", zstd_checksum=True)
              for c in _zarr.chunk_grid(big, 256, 256)]
    pid = service.register_zarr_plane(next(_ids), 0, 0, 0, pbx.UINT16, 512, 512, 256, 256, "blosc", chunks)
    assert np.array_equal(plane_be(service, pid, ">u2", 512, 512), big)
    service.release_plane(pid)
