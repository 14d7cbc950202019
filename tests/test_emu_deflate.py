"""The segment-deflate algorithm (the phases the HIP kernel runs), emulated on the CPU.

Checks RFC 1950/1951 validity with zlib's inflate, Adler-32 / CRC-32 combination math,
and compressed size against zlib level 6 (the reference's java.util.zip.Deflater).
"""
import zlib

import numpy as np
import pytest

import _emu


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 63, 64, 65, 100, 1000, 16383, 16384, 16385,
                               32768, 40000, 100003])
@pytest.mark.parametrize("kind", ["random", "zeros", "lowent", "periodic"])
def test_roundtrip(n, kind):
    rng = np.random.default_rng(n)
    if kind == "random":
        s = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    elif kind == "zeros":
        s = bytes(n)
    elif kind == "lowent":
        s = rng.integers(0, 4, n, dtype=np.uint8).tobytes()
    else:
        s = (bytes(range(97)) * (n // 97 + 1))[:n]
    z, segs = _emu.deflate(s, 97)
    assert zlib.decompress(z) == s
    # per-segment CRC-32 of the compressed bytes (used for the PNG IDAT CRC)
    pos = 2
    for g in segs:
        assert zlib.crc32(z[pos:pos + g.nbytes]) == g.crc
        pos += g.nbytes
    assert pos == len(z) - 4


def test_crc_nibble_step_forms_match_zlib():
    """k_frame_wave's CRC multiply (Horner over nibbles, x^4 in one step) and byte update equal
    zlib's bitwise multmodp / CRC update on 2 M seeded random pairs (operators x^(8n) among them)."""
    assert _emu.crc_fast_mismatches(2_000_000, 7) == 0


def test_rle_symbol_counts_closed_form():
    """k_huff's wave-level code-length RLE counts each run's symbols in closed form: equal to the
    emulator's loop (rle_nsyms) for every run length 1..320 of every code length 0..15."""
    assert _emu.rle_closed_mismatches() == 0


def test_crc_combine_matches_zlib():
    rng = np.random.default_rng(1)
    for la, lb in [(0, 5), (5, 0), (1, 1), (100, 3000), (17, 65537)]:
        a = rng.integers(0, 256, la, dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, lb, dtype=np.uint8).tobytes()
        assert _emu.crc_combine(zlib.crc32(a), zlib.crc32(b), lb) == zlib.crc32(a + b)


@pytest.mark.parametrize("kind,limit", [(2, 1.01), (1, 1.03)])
def test_ratio_vs_zlib6(oracle, kind, limit):
    """512x512 uint16 PNG stream: GPU deflate within 1% of zlib-6 on G_NOISE (the headline
    generator) and within 3% on G_FAKE (one repeated row: matches run across the waves'
    2 KiB sub-segments, so only the 33 segment boundaries cut the 258-byte match chain)."""
    t = oracle.gen_region(kind, oracle.UINT16, 0, 0, 512, 512)
    s = oracle.png_filter_stream(t, oracle.UINT16, 512, 512, 0).tobytes()
    z, _ = _emu.deflate(s, 1025)
    assert zlib.decompress(z) == s
    assert len(z) <= limit * len(zlib.compress(s, 6))


@pytest.mark.parametrize("filt", [1, 2, 3, 4, 5])
def test_filtered_streams(oracle, filt):
    t = oracle.gen_region(1, oracle.UINT8, 0, 0, 300, 80)
    s = oracle.png_filter_stream(t, oracle.UINT8, 300, 80, filt).tobytes()
    z, _ = _emu.deflate(s, 301)
    assert zlib.decompress(z) == s


@pytest.mark.parametrize("kind", ["random", "periodic", "rows", "runs"])
def test_lz77_records_cover_the_segment(kind):
    """LZ77 stage records (what k_lz77 writes and the GPU test compares): per segment the
    literals plus the match lengths cover exactly the segment's bytes, every match starts in
    its wave's sub-segment and ends inside the segment (a match may run on into the next
    wave's sub-segment, whose parse then starts at its end: no two matches overlap), uses a
    candidate distance (1, 2, one row) and pays."""
    rng = np.random.default_rng(3)
    rowlen = 301
    if kind == "random":
        s = rng.integers(0, 256, 50000, dtype=np.uint8).tobytes()
    elif kind == "periodic":
        s = (bytes(range(5)) * 20000)[:50000]
    elif kind == "rows":
        row = rng.integers(0, 256, rowlen, dtype=np.uint8).tobytes()
        s = (row * 200)[:50000]
    else:  # runs of random lengths (3..3000 bytes): many run across the waves' 2 KiB boundaries
        parts, n = [], 0
        while n < 50000:
            ln = int(rng.integers(3, 3000))
            parts.append(bytes([int(rng.integers(0, 256))]) * ln)
            n += ln
        s = b"".join(parts)[:50000]
    hist, mrec = _emu.lz77(s, rowlen)
    n = _emu.lib().pbxemu_nsegs(len(s))
    seg = (-(-len(s) // n) + 15) // 16 * 16
    nw, mw = _emu.lib().pbxemu_threads() // 64, 256
    for k in range(n):
        sl = min(seg, len(s) - k * seg)
        lits = int(hist[k][:256].sum())
        covered, prev_end = 0, 0
        for w in range(nw):
            for m in range(int(mrec[k][w])):
                pm = int(mrec[k][nw + w * mw + m])
                d = int(mrec[k][nw + nw * mw + w * mw + m]) + 1
                p, ln = pm & 0xFFFF, (pm >> 16) + 3
                assert w * 2048 <= p < min((w + 1) * 2048, sl) and p + ln <= sl
                assert p >= prev_end
                prev_end = p + ln
                assert d in (1, 2, rowlen)
                assert ln >= (3 if d <= 256 else 4 if d <= 4096 else 6)
                covered += ln
        assert lits + covered == sl
        assert hist[k][256] == 1  # end of block


def test_runs_across_wave_boundaries_roundtrip():
    """Runs of random lengths through the whole deflate emulator: matches carried across the
    waves' sub-segments decode to the input."""
    rng = np.random.default_rng(11)
    parts, n = [], 0
    while n < 200000:
        ln = int(rng.integers(1, 5000))
        parts.append(bytes([int(rng.integers(0, 256))]) * ln)
        n += ln
    s = b"".join(parts)[:200000]
    z, _ = _emu.deflate(s, 1025)
    assert zlib.decompress(z) == s
    assert len(z) <= 1.1 * len(zlib.compress(s, 6)) + 64


def skewed_block_stream(seed=7):
    """One Huffman block of full segments: bytes 0..127 in all but the last, 128..255 in
    the last, no repeats.  The block's code favours the first ones, so the last one's share
    of a Huffman-coded block would exceed its 16 KiB output buffer: the block must be
    stored."""
    import numpy as np
    L = _emu.lib()
    nblk, seg = L.pbxemu_blk_segs(), L.pbxemu_split_max()
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 128, (nblk - 1) * seg, dtype=np.uint8)
    b = rng.integers(128, 256, seg, dtype=np.uint8)
    return np.concatenate([a, b]).tobytes()


def test_segment_share_over_capacity_is_stored():
    data = skewed_block_stream()
    z, blks = _emu.deflate(data, 256)
    assert zlib.decompress(z) == data
    assert blks[0].btype == 0  # stored: a coded block would overflow the third segment


@pytest.mark.parametrize("n", [1, 16383, 16384 * 16, 16384 * 16 + 1, 524800, 1024 * 2049, 3_000_017])
def test_blocks_split_segments_evenly(n):
    """A tile's segments go to ceil(nseg / BLK) Huffman blocks of nearly equal size (at most
    BLK segments each, sizes differing by at most one segment): the 33 segments of a 512x512
    uint16 PNG make one block of 33 (three of 11 at a cap of 16)."""
    L = _emu.lib()
    blk, seg = L.pbxemu_blk_segs(), L.pbxemu_split_max()
    data = bytes((i * 7 + (i >> 9)) & 0xFF for i in range(n))
    z, blks = _emu.deflate(data, 1025)
    assert zlib.decompress(z) == data
    nseg = L.pbxemu_nsegs(n)
    assert len(blks) == -(-nseg // blk)
    assert sum(b.len for b in blks) == n
    n0 = -(-n // seg)
    seg_len = min(seg, (-(-n // n0) + 15) // 16 * 16)  # deflate_split: equal but the last
    counts = [-(-b.len // seg_len) for b in blks]
    assert sum(counts) == nseg
    assert max(counts) <= blk and max(counts) - min(counts) <= 1
    # the exact even split of block_seg0 (pbx_config.h): block j holds [j*nseg/nb, (j+1)*nseg/nb)
    nb = -(-nseg // blk)
    assert counts == [(j + 1) * nseg // nb - j * nseg // nb for j in range(nb)]
    if n == 524800:  # the headline tile: 33 segments
        assert nseg == 33
        if blk >= 33:
            assert counts == [33]
        elif blk == 16:
            assert counts == [11, 11, 11]


def test_div_rcp_exact():
    """div_rcp (the kernels' division by a host-computed reciprocal: segment -> tile, stream
    offset -> plane row) equals integer division for divisors up to 2^31 and any 32-bit n."""
    import ctypes
    L = _emu.lib()
    L.pbxemu_div_rcp.restype = ctypes.c_uint32
    L.pbxemu_div_rcp.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    rng = np.random.default_rng(11)
    ds = [1, 2, 3, 7, 16, 33, 1025, 1040, 2049, 4097, 65535, 65536, 99991, 2**24 + 1, 2**31 - 1, 2**31]
    ds += [int(x) for x in rng.integers(2, 2**31, 200)]
    for d in ds:
        ns = [0, 1, d - 1, d, d + 1, 2 * d - 1, 2**32 - 1, 2**32 - 2, 2**31]
        ns += [int(x) for x in rng.integers(0, 2**32, 200)] + [int(x) for x in rng.integers(0, 2**20, 50)]
        for n in ns:
            n &= 0xFFFFFFFF
            assert L.pbxemu_div_rcp(n, d) == n // d, (n, d)
