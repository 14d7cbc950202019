"""CPU oracle pinned against the golden fixtures and independent restatements (no GPU)."""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

import _numpy_ref

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(HERE, "manifest.json")))
CASES = MANIFEST["cases"]
T = MANIFEST["tile"]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def read(name):
    with open(os.path.join(HERE, name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_raw(oracle, case):
    raw = oracle.gen_region(case["kind"], case["pixel_type"], T["x"], T["y"], T["w"], T["h"]).tobytes()
    assert sha(raw) == case["raw_sha256"]
    assert raw == read(f"raw_{case['name']}.bin")
    assert raw == _numpy_ref.region(case["kind"], case["pixel_type"], T["x"], T["y"], T["w"], T["h"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_png(oracle, case):
    raw = read(f"raw_{case['name']}.bin")
    st, png = oracle.png_encode(np.frombuffer(raw, np.uint8), case["pixel_type"], T["w"], T["h"])
    if "png_status" in case:
        assert st == case["png_status"] == 404
        return
    assert st == 0 and sha(png) == case["png_sha256"] and png == read(f"png_{case['name']}.png")
    r, px, meta = oracle.png_decode(png)
    assert r == 0 and sha(px) == case["png_pil_pixels_sha256"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_tiff(oracle, case):
    raw = read(f"raw_{case['name']}.bin")
    st, tif = oracle.tiff_encode(np.frombuffer(raw, np.uint8), case["pixel_type"], T["w"], T["h"])
    assert st == 0 and sha(tif) == case["tif_sha256"] == sha(read(f"tif_{case['name']}.tif"))
    r, px, meta = oracle.tiff_decode(tif, len(raw))
    assert r == 0 and sha(px) == case["tif_tifffile_pixels_sha256"]
    assert meta["big_endian"] == 1 and meta["compression"] == 1


def test_known_answer_survey_sizes(oracle):
    """SURVEY.md §6 measured zlib-6 sizes of the filter-None streams: 3,670 and 390,443."""
    for kind, name, want in ((1, "fake", 3670), (2, "noise", 390443)):
        t = oracle.gen_region(kind, oracle.UINT16, 0, 0, 512, 512)
        s = oracle.png_filter_stream(t, oracle.UINT16, 512, 512, 0).tobytes()
        assert len(zlib.compress(s, 6)) == want == MANIFEST["u16_512_png"][name]["zlib6_len"]
        assert sha(s) == MANIFEST["u16_512_png"][name]["stream_sha256"]


def test_fake_known_values(oracle):
    """FakeReader: pixel = typeMin + x; boxes of 10 px on rows < 10 hold s, no, z, c, t."""
    g = lambda pt, x, y: oracle.lib().pbxo_gen_sample(1, 0, 7, 1, 2, 3, pt, x, y)
    assert g(oracle.UINT16, 123, 50) == 123
    assert g(oracle.INT16, 0, 50) == 0x8000          # -32768
    assert g(oracle.INT8, 130, 50) == 2               # -128 + 130
    assert [g(oracle.UINT8, x, 0) for x in (5, 15, 25, 35, 45, 55)] == [0, 7, 1, 2, 3, 55]
    assert g(oracle.FLOAT, 3, 20) == 0x40400000       # 3.0f


def test_get_tile_semantics(oracle):
    """TileRequestHandler.getTile restated: defaulting, bounds, format dispatch, type checks."""
    plane = oracle.gen_region(2, oracle.UINT16, 0, 0, 40, 30, big_endian=False)
    st, body, w, h = oracle.get_tile(plane, False, oracle.UINT16, 40, 30, 0, 0, 0, 0, oracle.FMT_RAW)
    assert st == 0 and (w, h) == (40, 30) and body == oracle.gen_region(2, oracle.UINT16, 0, 0, 40, 30).tobytes()
    assert oracle.get_tile(plane, False, oracle.UINT16, 40, 30, 1, 0, 0, 5, oracle.FMT_RAW)[0] == 404
    assert oracle.get_tile(plane, False, oracle.UINT16, 40, 30, 0, 0, 4, 4, oracle.FMT_UNKNOWN)[0] == 404
    plane32 = oracle.gen_region(2, oracle.FLOAT, 0, 0, 40, 30)
    assert oracle.get_tile(plane32, True, oracle.FLOAT, 40, 30, 0, 0, 4, 4, oracle.FMT_PNG)[0] == 404
    st, tif, _, _ = oracle.get_tile(plane32, True, oracle.FLOAT, 40, 30, 2, 2, 4, 4, oracle.FMT_TIF)
    r, px, meta = oracle.tiff_decode(tif, 64)
    assert st == 0 and r == 0 and meta["sample_format"] == 3


@pytest.mark.parametrize("filt", range(6))
def test_png_filters_roundtrip(oracle, filt):
    """Every filter (and the adaptive choice) unfilters to the same pixels."""
    for pt, w, h in ((oracle.UINT16, 37, 11), (oracle.UINT8, 1, 5), (oracle.INT16, 64, 3)):
        t = oracle.gen_region(2, pt, 5, 5, w, h)
        s = oracle.png_filter_stream(t, pt, w, h, filt).tobytes()
        # wrap into a PNG by hand and decode with the oracle decoder
        import struct
        def chunk(tp, d):
            return struct.pack(">I", len(d)) + tp + d + struct.pack(">I", zlib.crc32(tp + d))
        png = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8 * oracle.BPP[pt], 0, 0, 0, 0))
               + chunk(b"IDAT", zlib.compress(s)) + chunk(b"IEND", b""))
        r, px, _ = oracle.png_decode(png)
        want = bytearray(t.tobytes())
        if pt in (oracle.INT8, oracle.INT16):
            want[0::oracle.BPP[pt]] = bytes(b ^ 0x80 for b in want[0::oracle.BPP[pt]])
        assert r == 0 and px == bytes(want)


def test_filename_and_content_type(oracle):
    assert oracle.tile_filename(5, 1, 2, 3, 0, 512, 256, 128, None) == "image5_z1_c2_t3_x0_y512_w256_h128.bin"
    assert oracle.tile_filename(5, 1, 2, 3, 0, 0, 1, 1, "png").endswith(".png")
    assert oracle.content_type("png") == "image/png"
    assert oracle.content_type("tif") == "image/tiff"
    assert oracle.content_type(None) == oracle.content_type("jpg") == "application/octet-stream"


def test_grid_pixel_checker_catches_a_wrong_tile(oracle):
    """check_png_grid_pixels (used on every tile of the full-size GPU grids) accepts the
    oracle's own PNGs and names a tile whose pixels belong elsewhere in the grid."""
    bodies = []
    for i in range(6):
        t = oracle.gen_region(2, oracle.UINT16, (i % 3) * 64, (i // 3) * 32, 64, 32)
        bodies.append(bytes(oracle.png_encode(t, oracle.UINT16, 64, 32)[1]))
    assert oracle.check_png_grid_pixels(bodies, oracle.UINT16, 64, 32, 3, 0) == []
    bodies[4] = bodies[1]
    assert oracle.check_png_grid_pixels(bodies, oracle.UINT16, 64, 32, 3, 0) == [4]


def _np_tile_none(tile_be, pt, w, h):
    """The adaptive tile mode restated in numpy (oracle/pbx_oracle.c adaptive_tile_none): on the
    middle row, the best of Sub/Up/Avg/Paeth by sum |byte - prediction| against None by the sum
    over the byte planes (i mod bpp) & 1 of squared byte-value counts; None wins ties."""
    bpp = BPP_OF[pt]
    rb = w * bpp
    rows = np.asarray(tile_be, np.uint8).reshape(h, rb).astype(np.int64)
    if pt in (0, 2):  # int8 / int16: APNGWriter's sign flip of the most significant byte
        rows[:, 0::bpp] ^= 0x80
    rs = h // 2
    cur = rows[rs]
    up = rows[rs - 1] if rs > 0 else np.zeros(rb, np.int64)
    left = np.concatenate([np.zeros(bpp, np.int64), cur[:-bpp]])[:rb]
    ul = np.concatenate([np.zeros(bpp, np.int64), up[:-bpp]])[:rb]
    p = left + up - ul
    pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
    paeth = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
    preds = [left, up, (left + up) >> 1, paeth]
    sads = [int(np.abs(cur - q).sum()) for q in preds]
    fb = int(np.argmin(sads))
    resid = (cur - preds[fb]) & 0xFF
    plane = (np.arange(rb) % bpp) & 1

    def q2(v):
        return sum(int((np.bincount(v[plane == k], minlength=256) ** 2).sum()) for k in (0, 1))

    return q2(cur) >= q2(resid)


BPP_OF = [1, 1, 2, 2, 4, 4, 4, 8]


def test_adaptive_tile_mode(oracle):
    """The adaptive filter's tile mode: the C oracle against the numpy
    restatement above on synthetic and Poisson-like tiles; a None-mode tile's stream is the
    filter-None stream, and on Poisson-like 16-bit tiles (microscope counts) the adaptive stream
    deflates no larger than None, as it did not before the tile mode."""
    rng = np.random.default_rng(6)
    cases = []
    for kind in (1, 2):
        for pt, w, h in ((oracle.UINT16, 64, 9), (oracle.UINT8, 37, 5), (oracle.INT16, 33, 4),
                         (oracle.INT8, 100, 2), (oracle.UINT16, 1, 1), (oracle.UINT16, 128, 64)):
            cases.append((oracle.gen_region(kind, pt, 3, 7, w, h), pt, w, h))
    for lam in (3.0, 40.0, 400.0):
        v = rng.poisson(lam, (64, 128)).astype(">u2")
        cases.append((np.frombuffer(v.tobytes(), np.uint8).copy(), oracle.UINT16, 128, 64))
    modes = []
    for t, pt, w, h in cases:
        m = oracle.adaptive_tile_none(t, pt, w, h)
        assert m == _np_tile_none(t, pt, w, h), (pt, w, h)
        s = oracle.png_filter_stream(t, pt, w, h, 5)
        if m:
            assert s.tobytes() == oracle.png_filter_stream(t, pt, w, h, 0).tobytes()
        modes.append(m)
    assert modes[-3:] == [True, True, True]  # Poisson-like: filtering does not pay
    assert not modes[5]  # G_FAKE 128x64 uint16: its gradients pay for the filters
    for t, pt, w, h in cases[-3:]:
        a = len(zlib.compress(oracle.png_filter_stream(t, pt, w, h, 5).tobytes(), 6))
        n = len(zlib.compress(oracle.png_filter_stream(t, pt, w, h, 0).tobytes(), 6))
        assert a <= n
