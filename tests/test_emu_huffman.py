"""CPU emulator of the Huffman stage: valid, complete, length-limited canonical codes on
realistic and adversarial histograms (tests/_hists.py)."""
import numpy as np
import pytest

import _emu
import _hists


def kraft(lengths, maxbits):
    return sum(2 ** (maxbits - int(l)) for l in lengths if l)


@pytest.mark.parametrize("case", range(len(_hists.cases())))
def test_huffman_codes_valid(case):
    h = _hists.cases()[case]
    sl = _hists.stream_len(h)
    codes, info = _emu.huffman(h, sl, 1)
    btype, hdr_bits, data_bits, nbytes = (int(x) for x in info)
    assert btype in (0, 1, 2)
    assert nbytes <= 5 + sl  # never worse than a stored block
    if btype != 2:
        return
    ll = codes[:288] >> 16
    dl = codes[288:320] >> 16
    assert ll.max() <= 15 and dl.max() <= 15
    # every used symbol has a code; literal/length and distance codes are complete
    assert all(ll[s] > 0 for s in range(286) if h[s])
    assert all(dl[s] > 0 for s in range(30) if h[288 + s])
    assert kraft(ll, 15) == 2 ** 15
    assert kraft(dl, 15) == 2 ** 15
    # the data bits are the histogram's cost under these lengths (+ extra bits)
    leb = [0] * 257 + [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0] + [0, 0]
    deb = [0, 0, 0, 0] + [k // 2 for k in range(2, 28)] + [0, 0]
    cost = sum(int(h[s]) * (int(ll[s]) + leb[s]) for s in range(286))
    cost += sum(int(h[288 + s]) * (int(dl[s]) + deb[s]) for s in range(30))
    assert cost == data_bits


ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def header_code_lengths(codes):
    """(HLIT, HDIST, 19 code-length-code lengths) from a dynamic block's header words."""
    words = [int(x) for x in codes[320:]]
    pos = 0

    def get(n):
        nonlocal pos
        v = 0
        for i in range(n):
            w, b = divmod(pos, 32)
            v |= ((words[w] >> b) & 1) << i
            pos += 1
        return v

    get(1)
    assert get(2) == 2
    hlit, hdist, hclen = get(5) + 257, get(5) + 1, get(4) + 4
    cl = [0] * 19
    for i in range(hclen):
        cl[ORDER[i]] = get(3)
    return hlit, hdist, cl


def random_hists(seed, n=300):
    """Histograms whose code lengths, and so the code-length code's frequencies, are very
    uneven: random supports with geometric, Fibonacci-like and flat weights."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        h = np.zeros(320, np.uint64)
        k = int(rng.integers(2, 286))
        syms = rng.choice(286, k, replace=False)
        kind = int(rng.integers(0, 3))
        if kind == 0:
            w = np.floor(rng.geometric(rng.uniform(0.05, 0.9), k) ** rng.uniform(1, 4))
        elif kind == 1:
            w = np.array([1, 1] + [0] * (k - 2), np.float64)
            for i in range(2, k):
                w[i] = min(w[i - 1] + w[i - 2], 1e4)
            rng.shuffle(w)
        else:
            w = rng.integers(1, 50, k).astype(np.float64)
        w = np.floor(w * (rng.uniform(2000, 60000) / w.sum()))  # a block's symbol count
        h[syms] = np.maximum(w, 1).astype(np.uint64)
        nd = int(rng.integers(0, 30))
        if nd:
            h[288 + rng.choice(30, nd, replace=False)] = rng.integers(1, 1000, nd).astype(np.uint64)
            h[257 + rng.choice(28, 3)] += 1  # some length codes with the distances
        h[256] = 1
        out.append(h)
    return out


@pytest.mark.parametrize("seed", range(4))
def test_code_length_code_complete(seed):
    """The 19-symbol code-length code is complete and limited to 7 bits for any histogram.
    zlib's overflow repair counts every node deeper than the limit, internal ones included
    (trees.c gen_bitlen); counting leaves only left over-subscribed 7-bit codes ("invalid
    code lengths set") for trees with leaves two or more levels past the limit."""
    cases = random_hists(seed) + (_hists.cases() if seed == 0 else [])
    for h in cases:
        sl = 60000
        codes, info = _emu.huffman(h, sl, 0)
        if int(info[0]) != 2:
            continue
        _, _, cl = header_code_lengths(codes)
        assert max(cl) <= 7
        assert kraft(cl, 7) == 2 ** 7, cl
        ll = codes[:288] >> 16
        dl = codes[288:320] >> 16
        assert kraft(ll, 15) == 2 ** 15 and kraft(dl, 15) == 2 ** 15


def test_deep_overflow_subtile_decodes(oracle):
    """Regression: a 256x256 int32 tiled-TIFF edge tile (mostly zero padding) whose last
    Huffman block needs the 7-bit repair two levels deep; its zlib stream must inflate."""
    import zlib
    pt, T, sx, sy = 4, 256, 1100, 760
    bpp = oracle.BPP[pt]
    plane = oracle.gen_region(2, pt, 0, 0, sx, sy, big_endian=True)
    tile = np.frombuffer(oracle.extract_be(plane, True, pt, sx * bpp, 0, 0, sx, sy).tobytes(),
                         np.uint8).reshape(sy, sx * bpp)
    sub = np.zeros((T, T * bpp), np.uint8)
    part = tile[2 * T:3 * T, 3 * T * bpp:4 * T * bpp]
    sub[:part.shape[0], :part.shape[1]] = part
    raw = sub.tobytes()
    z, _ = _emu.deflate(raw, T * bpp)
    assert zlib.decompress(z) == raw
