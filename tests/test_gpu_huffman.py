"""GPU Huffman stage (k_huff, one wave per segment: round-parallel merge, wave-level code
lengths and code-length code) against the CPU emulator's sequential construction, word
for word, through the C-ABI test hook pbx_test_huffman."""
import ctypes

import numpy as np
import pytest

import _emu
import _hists
import pbx

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("which", ["hists", "random"])
def test_gpu_huffman_matches_emulator(service, which):
    """`random`: uneven histograms whose code-length codes need zlib's 7-bit overflow
    repair several levels deep (test_emu_huffman.random_hists)."""
    from test_emu_huffman import random_hists
    hs = (_hists.cases(seed=0) + _hists.cases(seed=1) if which == "hists"
          else random_hists(0, 200) + random_hists(2, 200))
    n = len(hs)
    hist = np.ascontiguousarray(np.stack(hs), dtype=np.uint32)
    sl_last = np.zeros((n, 2), np.uint32)
    for k, h in enumerate(hs):
        sl_last[k] = (_hists.stream_len(h), k & 1)
    codes = np.zeros((n, 480), np.uint32)
    info = np.zeros((n, 4), np.uint32)
    r = pbx.lib().pbx_test_huffman(service._h, hist.ctypes.data, sl_last.ctypes.data, n,
                                   codes.ctypes.data, info.ctypes.data)
    assert r == 0, pbx.lib().pbx_last_error()
    bad_cases = []
    for k in range(n):
        want_codes, want_info = _emu.huffman(hist[k], int(sl_last[k, 0]), int(sl_last[k, 1]))
        if list(info[k]) != list(want_info) or (codes[k] != want_codes).any():
            bad_cases.append((k, header_fields(codes[k]), header_fields(want_codes),
                              list(info[k]), list(want_info),
                              np.nonzero(codes[k][:320] != want_codes[:320])[0][:8].tolist()))
    assert not bad_cases, bad_cases[:4]


def header_fields(c):
    """BFINAL, BTYPE, HLIT, HDIST, HCLEN and the first code-length-code lengths."""
    v = int(c[320]) | (int(c[321]) << 32)
    f = [v & 1, (v >> 1) & 3, ((v >> 3) & 31) + 257, ((v >> 8) & 31) + 1, ((v >> 13) & 15) + 4]
    f.append([(v >> (17 + 3 * i)) & 7 for i in range(min(f[4], 15))])
    return f
