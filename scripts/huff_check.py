"""Diagnostic: run the GPU Huffman stage (pbx_test_huffman) repeatedly on the test
histograms and report mismatches against the CPU emulator."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _emu  # noqa: E402
import _hists  # noqa: E402
import pbx  # noqa: E402

ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def hdr(c):
    v = int(c[320]) | (int(c[321]) << 32) | (int(c[322]) << 64)
    hclen = ((v >> 13) & 15) + 4
    return [(v >> (17 + 3 * i)) & 7 for i in range(hclen)]


svc = pbx.PixelsService()
hs = _hists.cases(seed=0) + _hists.cases(seed=1)
n = len(hs)
hist = np.ascontiguousarray(np.stack(hs), dtype=np.uint32)
sl_last = np.array([(_hists.stream_len(h), k & 1) for k, h in enumerate(hs)], np.uint32)
want = [_emu.huffman(hist[k], int(sl_last[k, 0]), int(sl_last[k, 1])) for k in range(n)]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for rep in range(reps):
    codes = np.zeros((n, 480), np.uint32)
    info = np.zeros((n, 4), np.uint32)
    r = pbx.lib().pbx_test_huffman(svc._h, hist.ctypes.data, sl_last.ctypes.data, n,
                                   codes.ctypes.data, info.ctypes.data)
    assert r == 0
    bad = [k for k in range(n) if (codes[k] != want[k][0]).any() or (info[k] != want[k][1]).any()]
    print("rep", rep, "bad", bad, flush=True)
    for k in bad[:3]:
        print("  k", k, "gpu info", info[k].tolist(), "emu", want[k][1].tolist())
        print("  gpu cl", hdr(codes[k]))
        print("  emu cl", hdr(want[k][0]))
        d = np.nonzero(codes[k][:320] != want[k][0][:320])[0]
        print("  code diffs", d[:10].tolist())
