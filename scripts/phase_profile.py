"""Diagnostic: per-phase cycles of the deflate kernel (PBX_PHASE_PROFILE=1 build)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
os.environ.setdefault("PBX_PHASE_PROFILE", "1")
import pbx  # noqa: E402

gen = sys.argv[1] if len(sys.argv) > 1 else "noise"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
layout = sys.argv[3] if len(sys.argv) > 3 else "grid"  # "tall": one 512-px column of tiles
pt = pbx.UINT8 if len(sys.argv) > 4 and sys.argv[4] == "u8" else pbx.UINT16  # u8: configs[0]'s type
svc = pbx.PixelsService(device=0, stage_rows=os.environ.get("PBX_STAGE_ROWS", "0") == "1",
                       png_filter=int(os.environ.get("PBX_PNG_FILTER", "0")))
if layout == "tall":
    svc.register_plane(1, 0, 0, 0, pbx.UINT16, 512, 512 * 4096, generator=gen)
    ctxs = [pbx.TileCtx(1, 0, 0, 0, 0, i * 512, 512, 512, format="png") for i in range(n)]
elif layout == "same":  # every request the same tile: the plane reads hit the caches
    svc.register_plane(1, 0, 0, 0, pt, 32768, 32768, generator=gen)
    ctxs = [pbx.TileCtx(1, 0, 0, 0, 0, 0, 512, 512, format="png") for i in range(n)]
else:
    svc.register_plane(1, 0, 0, 0, pt, 32768, 32768, generator=gen)
    ctxs = [pbx.TileCtx(1, 0, 0, 0, (i % 64) * 512, (i // 64) * 512, 512, 512, format="png")
            for i in range(n)]
for _ in range(2):
    b = pbx.Batch(svc, ctxs)
    b.launch()
    b.sync()
    s = b.stats()
    print(gen, "deflate ms", round(s.ms_deflate, 3), "lz77", round(s.ms_lz77, 3), "huff",
          round(s.ms_huff, 3), "encode", round(s.ms_encode, 3), "frame", round(s.ms_assemble, 3),
          "segments", s.segments, "out", s.deflate_out_bytes, flush=True)
    b.close()
