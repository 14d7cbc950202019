"""GPU LZ77 stage (k_lz77: bit-parallel candidate masks, wave walk of paying positions,
wave-wide extension, interleaved literal histograms) against the CPU emulator's sequential
greedy/lazy parse (ph_parse_emu), segment by segment: the symbol histogram and every match
record must be identical.  Through the C-ABI test hook pbx_test_batch_lz77."""
import zlib

import numpy as np
import pytest

import _emu
import pbx

pytestmark = pytest.mark.gpu


def _streams():
    """(name, pixel type, w, h, plane array big-endian) cases that stress the parse: noise,
    long runs, row repeats, short periodic matches, rows longer than the window, tiny rows."""
    rng = np.random.default_rng(5)
    out = []
    yy, xx = np.mgrid[0:96, 0:700]
    out.append(("noise16", pbx.UINT16, rng.integers(0, 4096, (96, 700)).astype(">u2")))
    out.append(("runs8", pbx.UINT8, ((xx // 37) % 3 * 50 + (yy // 11) % 2).astype(np.uint8)))
    out.append(("period3", pbx.UINT8, (xx % 3 * 7 + (rng.random((96, 700)) < 0.05)).astype(np.uint8)))
    rows = np.tile(rng.integers(0, 65536, (1, 700)), (96, 1)).astype(">u2")
    rows[::7] = rng.integers(0, 65536, (14, 700))
    out.append(("rowrep16", pbx.UINT16, rows))
    out.append(("zeros16", pbx.UINT16, np.zeros((96, 700), ">u2")))
    wide = rng.integers(0, 3, (24, 2600)).astype(">u2")  # rowlen 5201 > the 4 KiB window
    wide[1::2] = wide[0::2]
    out.append(("wide16", pbx.UINT16, wide))
    out.append(("narrow8", pbx.UINT8, rng.integers(0, 2, (400, 3)).astype(np.uint8)))
    # the headline geometry (rows of whole 16-byte chunks: k_lz77's fast fill, three-row
    # blocks for 16-bit samples): 12-bit noise, and rows repeated in runs (matches extended
    # past the cap from the lanes' equality masks)
    out.append(("noise512", pbx.UINT16, rng.integers(0, 4096, (80, 512)).astype(">u2")))
    rep = np.repeat(rng.integers(0, 65536, (10, 512)), 8, axis=0).astype(">u2")
    rep[5::13] = rng.integers(0, 65536, (len(rep[5::13]), 512))
    out.append(("rowrep512", pbx.UINT16, rep))
    # one run over whole segments (k_lz77's predicted wave starts right), and the same run
    # broken at a few random pixels (predictions wrong from some wave on: serial rounds)
    out.append(("zeros512", pbx.UINT16, np.zeros((80, 512), ">u2")))
    brk = np.full((80, 512), 0x1234, ">u2")
    brk.flat[rng.choice(80 * 512, 40, replace=False)] = rng.integers(0, 65536, 40)
    out.append(("runbreak512", pbx.UINT16, brk))
    # runs of random lengths (1..3000 samples) laid row after row: predictions right and
    # wrong at random waves, carries of every length
    vals, n = [], 0
    while n < 80 * 512:
        ln = int(rng.integers(1, 3000))
        vals.append(np.full(ln, int(rng.integers(0, 65536)), np.uint16))
        n += ln
    out.append(("randruns512", pbx.UINT16, np.concatenate(vals)[:80 * 512].reshape(80, 512).astype(">u2")))
    return out


@pytest.mark.parametrize("case", range(12))
def test_gpu_lz77_matches_emulator(service, case):
    name, pt, a = _streams()[case]
    h, w = a.shape
    iid = 9_500_000 + case
    if name.endswith("512"):  # little-endian plane: the byte-swapping fill (the headline's)
        service.register_plane(iid, 0, 0, 0, pt, w, h, data=a.astype("<u2"), big_endian=False)
    else:
        service.register_plane(iid, 0, 0, 0, pt, w, h, data=a, big_endian=True)
    b = pbx.Batch(service, [pbx.TileCtx(iid, 0, 0, 0, 0, 0, w, h, format="png")])
    b.launch()
    b.sync()
    nseg = b.stats().segments
    L = _emu.lib()
    gh, gm = b.lz77_records(nseg, L.pbxemu_hist_words(), L.pbxemu_mrec_words())
    b.close()
    bpp = pbx.BYTES_PER_PIXEL[pt]
    raw = a.tobytes()
    stream = b"".join(b"\x00" + raw[r * w * bpp:(r + 1) * w * bpp] for r in range(h))
    eh, em = _emu.lz77(stream, 1 + w * bpp)
    assert gh.shape == eh.shape
    nw = L.pbxemu_threads() // 64

    def records(m, wv):  # (position, length, distance) of wave wv's kept matches
        n = int(m[wv])
        return [(int(m[nw + wv * 256 + j]) & 0xFFFF, (int(m[nw + wv * 256 + j]) >> 16) + 3,
                 int(m[nw + nw * 256 + wv * 256 + j]) + 1) for j in range(n)]

    for k in range(nseg):
        for wv in range(nw):  # the match records first: they say where a difference starts
            g, e = records(gm[k], wv), records(em[k], wv)
            assert g == e, (name, k, wv, [x for x in g if x not in e][:4], [x for x in e if x not in g][:4])
        assert (gh[k] == eh[k]).all(), (name, k, np.nonzero(gh[k] != eh[k])[0][:8],
                                        gh[k][gh[k] != eh[k]][:8], eh[k][gh[k] != eh[k]][:8])


def _records(m, nw, wv):
    n = int(m[wv])
    return [(int(m[nw + wv * 256 + j]) & 0xFFFF, (int(m[nw + wv * 256 + j]) >> 16) + 3,
             int(m[nw + nw * 256 + wv * 256 + j]) + 1) for j in range(n)]


@pytest.mark.parametrize("filt", [1, 2, 4, 5])
@pytest.mark.parametrize("kind", ["ramp", "ramp_broken"])
def test_gpu_lz77_filtered_ramp_rows(oracle, filt, kind):
    """Row-filtered FakeReader ramps: Up and the adaptive choice turn
    every row into the filter byte and a run of zeros, Sub into the first sample and a period-2
    run, so every run breaks at each row's filter byte and k_lz77's predicted wave starts (a
    258-byte chain from the segment start) are wrong in nearly every wave: the repair rounds
    must still give the serial parse's records exactly."""
    rng = np.random.default_rng(11 + filt)
    w, h = 512, 96
    a = np.tile((np.arange(w) + 300).astype(np.uint16), (h, 1))
    if kind == "ramp_broken":  # a few pixels and whole rows off the ramp
        a.flat[rng.choice(w * h, 24, replace=False)] = rng.integers(0, 65536, 24)
        a[rng.choice(h, 5, replace=False)] = rng.integers(0, 65536, (5, w))
    with pbx.PixelsService(png_filter=filt) as svc:
        iid = 9_600_000 + filt
        svc.register_plane(iid, 0, 0, 0, pbx.UINT16, w, h, data=a.astype("<u2"), big_endian=False)
        b = pbx.Batch(svc, [pbx.TileCtx(iid, 0, 0, 0, 0, 0, w, h, format="png")])
        b.launch()
        b.sync()
        nseg = b.stats().segments
        L = _emu.lib()
        gh, gm = b.lz77_records(nseg, L.pbxemu_hist_words(), L.pbxemu_mrec_words())
        b.close()
    tile_be = np.frombuffer(a.astype(">u2").tobytes(), np.uint8)
    stream = oracle.png_filter_stream(tile_be, pbx.UINT16, w, h, filt).tobytes()
    eh, em = _emu.lz77(stream, 1 + w * 2)
    assert gh.shape == eh.shape
    nw = L.pbxemu_threads() // 64
    carried = 0
    for k in range(nseg):
        for wv in range(nw):
            g, e = _records(gm[k], nw, wv), _records(em[k], nw, wv)
            assert g == e, (kind, filt, k, wv, [x for x in g if x not in e][:4], [x for x in e if x not in g][:4])
            carried += bool(e) and e[-1][0] + e[-1][1] > (wv + 1) * 2048
        assert (gh[k] == eh[k]).all(), (kind, filt, k, np.nonzero(gh[k] != eh[k])[0][:8])
    if kind == "ramp":
        assert carried >= nseg  # matches do run across the wave boundaries here


@pytest.mark.parametrize("boundary", [1, 3, 6])
@pytest.mark.parametrize("run", [3, 4])
def test_gpu_lz77_short_rowup_run_at_wave_boundary(service, boundary, run):
    """Rows of <= 256 bytes (row-up distance <= 256: a 3-byte match pays) with a row-up run of
    exactly `run` bytes ending at a sub-segment's last byte and going on for 45 more: the
    serial parse takes the 3-byte match there and extends it across the boundary, so k_lz77's
    boundary test must count a 3-byte row-up run as reachable (a 4-byte test missed it and the
    next wave parsed the run on its own)."""
    a, stream, e = _short_rowup_case(boundary, run)
    h, w = a.shape
    iid = 9_700_000 + 10 * boundary + run
    service.register_plane(iid, 0, 0, 0, pbx.UINT8, w, h, data=a, big_endian=True)
    b = pbx.Batch(service, [pbx.TileCtx(iid, 0, 0, 0, 0, 0, w, h, format="png")])
    b.launch()
    b.sync()
    nseg = b.stats().segments
    L = _emu.lib()
    gh, gm = b.lz77_records(nseg, L.pbxemu_hist_words(), L.pbxemu_mrec_words())
    b.close()
    eh, em = _emu.lz77(stream, 1 + w)
    nw = L.pbxemu_threads() // 64
    ew = _records(em[0], nw, boundary - 1)
    assert ew and ew[-1][0] == e - run and ew[-1][0] + ew[-1][1] > e  # the carried match
    for k in range(nseg):
        for wv in range(nw):
            g, x = _records(gm[k], nw, wv), _records(em[k], nw, wv)
            assert g == x, (boundary, run, k, wv, [y for y in g if y not in x][:4], [y for y in x if y not in g][:4])
        assert (gh[k] == eh[k]).all(), (boundary, run, k, np.nonzero(gh[k] != eh[k])[0][:8])


def _short_rowup_case(boundary, run, w=100, h=400):
    """uint8 noise (rowlen w + 1) whose stream bytes [e - run, e + 45) equal the row above's
    (e = 2048 boundary) and byte e - run - 1 does not; returns (pixels, PNG stream, e)."""
    rng = np.random.default_rng(100 * boundary + run)
    a = rng.integers(0, 256, (h, w)).astype(np.uint8)
    rl = w + 1
    e = 2048 * boundary
    assert (e - run - 1) % rl != 0  # the byte before the run is a pixel, not a filter byte
    for p in range(e - run, e + 45):  # in stream order: row-up sources are final
        if p % rl:
            a[p // rl, p % rl - 1] = a[p // rl - 1, p % rl - 1]
    q = e - run - 1
    a[q // rl, q % rl - 1] = (int(a[q // rl - 1, q % rl - 1]) + 1) % 256
    raw = a.tobytes()
    stream = b"".join(b"\x00" + raw[i * w:(i + 1) * w] for i in range(h))
    assert stream[e - run:e + 45] == stream[e - run - rl:e + 45 - rl] and stream[q] != stream[q - rl]
    return a, stream, e



def _structured_stream(rng, rowbytes, h, ncopies):
    """A filter-None PNG stream (h rows of rowbytes + 1 bytes) with random runs: ncopies forward
    copies of random length (3..300) at distance 1, 2 or one row, at random places (filter
    bytes stay 0, so a copy over one breaks there); returns (row bytes (h, rowbytes), stream)."""
    rl = rowbytes + 1
    s = bytearray(rng.integers(0, 256, h * rl).astype(np.uint8).tobytes())
    for r in range(h):
        s[r * rl] = 0
    for _ in range(ncopies):
        d = [1, 2, rl][int(rng.integers(3))]
        p = int(rng.integers(d, len(s)))
        ln = int(rng.integers(3, 301))
        for q in range(p, min(p + ln, len(s))):
            if q % rl:
                s[q] = s[q - d]
    return np.frombuffer(bytes(s), np.uint8).reshape(h, rl)[:, 1:].copy(), bytes(s)


@pytest.mark.parametrize("seed", range(12))
def test_gpu_lz77_structured_fuzz(service, seed):
    """Random tiles of random row lengths (4..8401 bytes: row-up distance above and below the
    256-byte and 4 KiB thresholds of match_minlen) full of runs at distances 1, 2 and one row
    landing anywhere -- across sub-segment and segment boundaries, filter bytes, the window --
    as big-endian 8-bit planes and little-endian 16-bit ones (the byte-swapping fill): every
    segment's records and histogram equal the emulator's serial parse."""
    rng = np.random.default_rng(7000 + seed)
    L = _emu.lib()
    nw = L.pbxemu_threads() // 64
    for t in range(8):
        w = int(rng.choice([3, 17, 100, 255, 256, 300, 511, 700, 2047, 4095, 4200]))
        bpp = 1 + t % 2
        h = max(3, int(rng.integers(20000, 80000)) // (w * bpp + 1))
        rows, stream = _structured_stream(rng, w * bpp, h, int(rng.integers(20, 400)))
        iid = 9_800_000 + 100 * seed + t
        if bpp == 1:
            service.register_plane(iid, 0, 0, 0, pbx.UINT8, w, h, data=rows, big_endian=True)
        else:
            a = rows.view(">u2").astype("<u2")
            service.register_plane(iid, 0, 0, 0, pbx.UINT16, w, h, data=a, big_endian=False)
        b = pbx.Batch(service, [pbx.TileCtx(iid, 0, 0, 0, 0, 0, w, h, format="png")])
        b.launch()
        b.sync()
        nseg = b.stats().segments
        gh, gm = b.lz77_records(nseg, L.pbxemu_hist_words(), L.pbxemu_mrec_words())
        b.close()
        eh, em = _emu.lz77(stream, w * bpp + 1)
        assert gh.shape == eh.shape
        for k in range(nseg):
            for wv in range(nw):
                g, x = _records(gm[k], nw, wv), _records(em[k], nw, wv)
                assert g == x, (seed, t, w, h, k, wv, [y for y in g if y not in x][:4], [y for y in x if y not in g][:4])
            assert (gh[k] == eh[k]).all(), (seed, t, w, h, k, np.nonzero(gh[k] != eh[k])[0][:8])


def _structured_rows(rng, rowbytes, h, ncopies):
    """numpy form of _structured_stream for larger cases: runs at distance 1 / 2 (pattern
    fills) and one row (slice copies of at most a row), filter bytes zeroed afterwards."""
    rl = rowbytes + 1
    s = rng.integers(0, 256, h * rl).astype(np.uint8)
    for _ in range(ncopies):
        d = [1, 2, rl][int(rng.integers(3))]
        p = int(rng.integers(d, s.size))
        ln = min(int(rng.integers(3, 301)), s.size - p)
        if d < 3:
            s[p:p + ln] = np.resize(s[p - d:p], ln)
        else:
            ln = min(ln, rl)
            s[p:p + ln] = s[p - d:p - d + ln]
    s[::rl] = 0
    return s.reshape(h, rl)[:, 1:].copy(), s.tobytes()


@pytest.mark.parametrize("filt", [0, 5])
@pytest.mark.parametrize("seed", range(4))
def test_gpu_png_structured_fuzz_bytes(oracle, seed, filt):
    """End to end on run-structured data: 320 tiles of random heights in one batch (more
    Huffman blocks than the small-batch k_huff takes: the batch kernels), 8- and 16-bit
    planes of row lengths across match_minlen's thresholds -- every tile's zlib stream equals
    the emulator's deflate byte for byte and inflates to the tile's scanlines, and its PNG
    chunks carry valid CRCs (zlib.crc32 over type + data).  With the adaptive row filter (filt 5:
    the row-filtered k_lz77 variant, its VALU walk and row-start predictions) the emulator deflates
    the GPU's own filtered scanlines and the PNG decodes to the plane's pixels."""
    with pbx.PixelsService(png_filter=filt) as service:
        _png_structured_fuzz(service, oracle, seed, filt)


def _png_structured_fuzz(service, oracle, seed, filt):
    rng = np.random.default_rng(8100 + seed)
    ctxs, streams = [], []
    for wi, w in enumerate([3, 100, 256, 300, 700, 2100]):
        bpp = 1 + wi % 2
        hs = [max(1, int(rng.integers(2000, 40000)) // (w * bpp + 1)) for _ in range(320 // 6 + 1)]
        rows, stream = _structured_rows(rng, w * bpp, sum(hs), 60 * len(hs))
        iid = 9_900_000 + 1000 * filt + 100 * seed + wi
        if bpp == 1:
            service.register_plane(iid, 0, 0, 0, pbx.UINT8, w, sum(hs), data=rows, big_endian=True)
        else:
            service.register_plane(iid, 0, 0, 0, pbx.UINT16, w, sum(hs), data=rows.view(">u2").astype("<u2"),
                                   big_endian=False)
        y = 0
        for h in hs:
            ctxs.append(pbx.TileCtx(iid, 0, 0, 0, 0, y, w, h, format="png"))
            rl = w * bpp + 1
            streams.append((stream[y * rl:(y + h) * rl], rl, rows[y:y + h].tobytes(), w, h, bpp))
            y += h
    res = service.get_tiles(ctxs)
    for i, ((st, body), (stream, rl, px, w, h, bpp)) in enumerate(zip(res, streams)):
        assert st == pbx.OK, i
        if filt:  # the GPU's filtered scanlines; the pixels must come back exactly
            n = int.from_bytes(body[91:95], "big")  # IDAT length
            stream = zlib.decompress(body[99:95 + n + 4])
            r, dpx, _ = oracle.png_decode(body)
            assert r == 0 and dpx == px, (seed, i)
        z, _ = _emu.deflate(stream, rl)
        assert body[99:99 + len(z)] == z, (seed, i, rl, len(stream))
        assert zlib.decompress(z) == stream
        o = 8
        while o < len(body):  # every chunk: length, type, data, CRC-32 of type + data
            n = int.from_bytes(body[o:o + 4], "big")
            assert zlib.crc32(body[o + 4:o + 8 + n]) == int.from_bytes(body[o + 8 + n:o + 12 + n], "big"), (i, body[o + 4:o + 8])
            o += 12 + n
        assert o == len(body) and body[-8:-4] == b"IEND"
