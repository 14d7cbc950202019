"""Row f3 alone: the 6-level resolution pyramid of the headline's 32768^2 uint16 G_NOISE plane
(bench.py's pyramid line), three builds; prints the kernel ms (HIP events) and the HBM
fraction of the algorithmic bytes (every level read once, every lower level written once).
$PBX_LIB selects the library (A/B of k_downsample forms)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import pbx  # noqa: E402

side = 32768
pb, wl = 0, side
for _ in range(6):
    pb += 2 * wl * wl + 2 * ((wl + 1) // 2) ** 2
    wl = (wl + 1) // 2
ms = []
for k in range(4):
    with pbx.PixelsService(device=0) as svc:
        pid = svc.register_plane(5, 0, 0, 0, pbx.UINT16, side, side, generator="noise")
        _, t = svc.build_pyramid(pid, 6, timing=True)
        if k:
            ms.append(t)
m = sum(ms) / len(ms)
print(f"pyramid ms {m:.3f} ({' '.join(f'{x:.3f}' for x in ms)}) frac {pb / (m * 1e-3) / 1e9 / 8000:.4f}", flush=True)
