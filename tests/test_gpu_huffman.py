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


def _block_len(h):
    """Stream bytes of a whole block's histogram (literals + 3 bytes per match)."""
    return int(h[:256].sum()) + 3 * int(h[257:286].sum())


@pytest.mark.parametrize("which", ["hists", "random", "block"])
def test_gpu_huffman_matches_emulator(service, which):
    """`random`: uneven histograms whose code-length codes need zlib's 7-bit overflow
    repair several levels deep (test_emu_huffman.random_hists).  `block`: the histograms
    of whole blocks (11 segments; the headline's 512x512 uint16 tiles make one of 33): symbol counts
    far above 65535, so the merge's internal weights need 32 bits."""
    from test_emu_huffman import random_hists
    if which == "hists":
        hs = _hists.cases(seed=0) + _hists.cases(seed=1)
    elif which == "random":
        hs = random_hists(0, 200) + random_hists(2, 200)
    else:
        hs = [h * 11 for h in _hists.cases(seed=0) + random_hists(4, 100)]
    n = len(hs)
    hist = np.ascontiguousarray(np.stack(hs), dtype=np.uint32)
    sl_last = np.zeros((n, 2), np.uint32)
    for k, h in enumerate(hs):
        sl_last[k] = (_block_len(h) if which == "block" else _hists.stream_len(h), k & 1)
    codes = np.zeros((n, 480), np.uint32)
    info = np.zeros((n, 4), np.uint32)
    r = pbx.lib().pbx_test_huffman(service._h, hist.ctypes.data, sl_last.ctypes.data, n,
                                   codes.ctypes.data, info.ctypes.data)
    assert r == 0, pbx.lib().pbx_last_error()
    bad_cases = []
    for k in range(n):
        want_codes, want_info = _emu.huffman(hist[k], int(sl_last[k, 0]), int(sl_last[k, 1]))
        # (block: the codes only -- the test hook's block is ONE segment, which k_huff then
        # stores because its share exceeds k_encode's segment buffer; the emulator's hook
        # has no such rule)
        info_ok = which == "block" or list(info[k]) == list(want_info)
        if not info_ok or (codes[k] != want_codes).any():
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
