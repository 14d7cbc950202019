"""Compressed size of 512x512 uint16 filter-None PNG streams under zlib levels/strategies and
under this repo's deflate (the CPU emulator of the GPU phases, byte-identical to the GPU):
the DESIGN.md section 2 table.  CPU only: python scripts/zlib_levels.py"""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _emu  # noqa: E402
import _oracle as O  # noqa: E402

T = 512


def stream(tile_be):
    rows = np.frombuffer(tile_be, np.uint8).reshape(T, 2 * T)
    return np.concatenate([np.zeros((T, 1), np.uint8), rows], 1).tobytes()


def poisson_tiles():
    # the bench's Poisson-like plane (bench.adaptive_filter_line): lambda drifting 200..300
    rng = np.random.default_rng(1234)
    ps = 8192
    yy, xx = np.mgrid[0:ps:64, 0:ps:64]
    lam = 200.0 + 100.0 * (0.5 + 0.25 * np.sin(xx / 900.0) + 0.25 * np.cos(yy / 1300.0))
    pois = rng.poisson(np.repeat(np.repeat(lam, 64, 0), 64, 1)).astype(np.uint16)
    for j in range(8):
        x, y = (j * 7 % (ps // T)) * T, (j * 5 % (ps // T)) * T
        yield pois[y:y + T, x:x + T].astype(">u2").tobytes()


def gen_tiles(kind):
    for j in range(8):
        x, y = (j * 7 % 64) * T, (j * 5 % 64) * T
        yield O.gen_region(kind, O.UINT16, x, y, T, T).tobytes()


MODES = [("zlib6", 6, 0), ("zlib9", 9, 0), ("zlib1", 1, 0), ("huffman_only", 6, zlib.Z_HUFFMAN_ONLY)]
for name, tiles in (("noise", gen_tiles(2)), ("fake", gen_tiles(1)), ("poisson", poisson_tiles())):
    tot, n = {}, 0
    for t in tiles:
        s = stream(t)
        n += 1
        for m, lv, st in MODES:
            c = zlib.compressobj(lv, zlib.DEFLATED, 15, 8, st)
            tot[m] = tot.get(m, 0) + len(c.compress(s) + c.flush())
        z, _ = _emu.deflate(s, 2 * T + 1)
        assert zlib.decompress(z) == s
        tot["here"] = tot.get("here", 0) + len(z)
    print(name, {k: round(v / n, 1) for k, v in tot.items()},
          "here vs zlib6: %+.1f%%" % (100.0 * (tot["here"] / tot["zlib6"] - 1)))
