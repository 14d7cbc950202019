"""Diagnostic: tiled deflate-TIFF sub-tile streams vs the CPU emulation (which tile, which
segment, first differing byte).  python scripts/diag_tiled.py [T] [pixel_type]"""
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "omero-ms-pixel-buffer_amd")]
import numpy as np  # noqa: E402
import pbx  # noqa: E402
import _emu  # noqa: E402
import _oracle  # noqa: E402
from test_tiff_tiled import _tile_table  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 256
pt = int(sys.argv[2]) if len(sys.argv) > 2 else pbx.INT32
O = _oracle
O.lib()
sx, sy = 1100, 760
bpp = O.BPP[pt]
plane = O.gen_region(2, pt, 0, 0, sx, sy, big_endian=True)
with pbx.PixelsService(tiff_tile=T, tiff_deflate=True) as svc:
    svc.register_plane(1, 0, 0, 0, pt, sx, sy, data=plane, big_endian=True)
    (st, body), = svc.get_tiles([pbx.TileCtx(1, 0, 0, 0, 0, 0, 0, 0, format="tif")])
print("status", st, "bytes", len(body))
tile = O.extract_be(plane, True, pt, sx * bpp, 0, 0, sx, sy)
tile = np.frombuffer(tile.tobytes(), np.uint8).reshape(sy, sx * bpp)
offs, cnts = _tile_table(body)
nx = (sx + T - 1) // T
bad = 0
for k, (o, c) in enumerate(zip(offs, cnts)):
    ty, tx = divmod(k, nx)
    sub = np.zeros((T, T * bpp), np.uint8)
    part = tile[ty * T:(ty + 1) * T, tx * T * bpp:(tx + 1) * T * bpp]
    sub[:part.shape[0], :part.shape[1]] = part
    raw = sub.tobytes()
    z, blks = _emu.deflate(raw, T * bpp)
    g = body[o:o + c]
    ok = g == z
    try:
        dec = zlib.decompress(g) == raw
    except zlib.error as e:
        dec = str(e)
    if not ok or dec is not True:
        bad += 1
        i = next((i for i in range(min(len(g), len(z))) if g[i] != z[i]), min(len(g), len(z)))
        segs = [(b.nbytes, b.btype, b.len) for b in blks]
        print(f"tile {k} ({tx},{ty}) gpu {len(g)} emu {len(z)} first diff at {i} decode {dec}")
        acc = 2
        for j, (nb, bt, ln) in enumerate(segs):
            print(f"   seg {j} emu bytes [{acc},{acc + nb}) btype {bt} len {ln}")
            acc += nb
print("bad tiles", bad, "of", len(offs))
