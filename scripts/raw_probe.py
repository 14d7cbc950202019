"""k_extract alone: the headline grid (4096 x 512^2 uint16 of the 32768^2 G_NOISE plane) as raw
tiles, aligned (x = 512 i) and unaligned (x = 512 i + 3, x * bpp mod 16 = 6), one kernel
stream; prints the mean k_extract HIP-event time and GB/s (2 x tile bytes) over `n` batches.
$PBX_EXT_BLK sets the bytes per workgroup (runtime.cpp ext_blk_bytes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import pbx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
svc = pbx.PixelsService(device=0)
svc.set_kernel_streams(1, 0)
svc.register_plane(1, 0, 0, 0, pbx.UINT16, 32768, 32768, generator="noise")
for name, dx in (("aligned", 0), ("unaligned", 3)):
    ctxs = [pbx.TileCtx(1, 0, 0, 0, (i % 64) * 512 + (dx if i % 64 < 63 else -5 if dx else 0),
                        (i // 64) * 512, 512, 512) for i in range(4096)]
    reqs = pbx.make_reqs(ctxs)
    ms = []
    for k in range(n + 1):
        b = pbx.Batch(svc, reqs=reqs)
        b.launch()
        b.sync()
        s = b.stats()
        if k:
            ms.append(s.ms_extract)
        b.close()
    m = sum(ms) / len(ms)
    print(f"{name} ext_blk={os.environ.get('PBX_EXT_BLK', 16384)} k_extract {m:.3f} ms "
          f"{2 * s.in_bytes / (m * 1e-3) / 1e9:.1f} GB/s", flush=True)
svc.close()
