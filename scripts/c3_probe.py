"""configs[2]'s batch alone (4096 x 1024^2 uint16 G_NOISE tiles -> PNG from a 65536^2 plane),
one kernel stream, n batches: per-kernel HIP-event times (the A/B workload for that line)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import pbx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
svc = pbx.PixelsService(device=0)
svc.register_plane(3, 0, 0, 0, pbx.UINT16, 65536, 65536, generator="noise")
ctxs = [pbx.TileCtx(3, 0, 0, 0, (i % 64) * 1024, (i // 64) * 1024, 1024, 1024, format="png") for i in range(4096)]
reqs = pbx.make_reqs(ctxs)
for _ in range(n):
    b = pbx.Batch(svc, reqs=reqs)
    b.launch()
    b.sync()
    s = b.stats()
    print("c3 deflate ms", round(s.ms_deflate, 3), "lz77", round(s.ms_lz77, 3), "huff", round(s.ms_huff, 3),
          "encode", round(s.ms_encode, 3), "out", s.deflate_out_bytes, flush=True)
    b.close()
svc.close()
