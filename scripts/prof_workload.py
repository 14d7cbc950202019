"""Profiling workload: the bench's batch (4096 x 512^2 uint16 G_NOISE tiles -> PNG), run
`n` times (default 3), no phase stamps; $PBX_PW_FILTER picks the PNG filter (default None).  Used under rocprofv3 (kernel trace / PMC)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import pbx  # noqa: E402

gen = sys.argv[1] if len(sys.argv) > 1 else "noise"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
svc = pbx.PixelsService(device=0, png_filter=int(os.environ.get("PBX_PW_FILTER", "0")))
svc.register_plane(1, 0, 0, 0, pbx.UINT16, 32768, 32768, generator=gen)
ctxs = [pbx.TileCtx(1, 0, 0, 0, (i % 64) * 512, (i // 64) * 512, 512, 512, format="png")
        for i in range(4096)]
reqs = pbx.make_reqs(ctxs)
for _ in range(n):
    b = pbx.Batch(svc, reqs=reqs)
    b.launch()
    b.sync()
    s = b.stats()
    print(gen, "deflate ms", round(s.ms_deflate, 3), "lz77", round(s.ms_lz77, 3), "huff",
          round(s.ms_huff, 3), "encode", round(s.ms_encode, 3), "filter ms", round(s.ms_filter, 3),
          "out", s.deflate_out_bytes, flush=True)
    b.close()
svc.close()
