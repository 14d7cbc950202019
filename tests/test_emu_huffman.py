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
