"""Diagnostic: one blosc-lz4 Zarr plane through the PBX_ZARR_DIAG build (stream 0's clocks)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "omero-ms-pixel-buffer_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import pbx, _oracle as O, _zarr
side, ch = 2048, 512
plane = O.gen_region(2, O.UINT16, 0, 0, side, side).view("<u2").reshape(side, side)
chunks = []
for cy in range(side // ch):
    for cx in range(side // ch):
        c = np.ascontiguousarray(plane[cy*ch:(cy+1)*ch, cx*ch:(cx+1)*ch])
        chunks.append(_zarr.cblosc_encode(c.tobytes(), 2, "lz4", 5, 2))
svc = pbx.PixelsService(device=0)
pid = svc.register_zarr_plane(1, 0, 0, 0, pbx.UINT16, side, side, ch, ch, "blosc", chunks, big_endian=False)
print("ok", pid, flush=True)
