"""Diagnostic: one zlib-1 Zarr plane through the PBX_ZARR_DIAG build (stream 0's clocks)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "omero-ms-pixel-buffer_amd"), os.path.join(ROOT, "tests")]
import numpy as np, zlib
import pbx, _oracle as O
side, ch = 2048, 512
plane = O.gen_region(2, O.UINT16, 0, 0, side, side).view("<u2").reshape(side, side)
chunks, offs = [], [0]
for cy in range(side // ch):
    for cx in range(side // ch):
        b = zlib.compress(np.ascontiguousarray(plane[cy*ch:(cy+1)*ch, cx*ch:(cx+1)*ch]).tobytes(), 1)
        chunks.append(b); offs.append(offs[-1] + len(b))
svc = pbx.PixelsService(device=0)
pid = svc.register_zarr_plane(1, 0, 0, 0, pbx.UINT16, side, side, ch, ch, "zlib", chunks, big_endian=False)
print("ok", pid, flush=True)
