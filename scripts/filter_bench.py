"""PNG filter kernels alone: 4096 x 512^2 uint16 G_NOISE tiles with each PNG filter (Sub, Up,
Avg, Paeth, adaptive), serial kernel stream; prints the filter kernel's HIP-event ms and its
HBM rate (tile bytes read + filtered stream written).  PBX_FILTER3=0 selects k_filter2."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import pbx  # noqa: E402

side = 32768
names = {1: "sub", 2: "up", 3: "avg", 4: "paeth", 5: "adaptive"}
for f in [int(a) for a in sys.argv[1:]] or [1, 2, 3, 4, 5]:
    with pbx.PixelsService(device=0, png_filter=f) as svc:
        svc.set_kernel_streams(1, 0)
        svc.register_plane(1, 0, 0, 0, pbx.UINT16, side, side, generator="noise")
        ctxs = [pbx.TileCtx(1, 0, 0, 0, (i % 64) * 512, (i // 64) * 512, 512, 512, format="png")
                for i in range(4096)]
        reqs = pbx.make_reqs(ctxs)
        ms = []
        for k in range(4):
            b = pbx.Batch(svc, reqs=reqs)
            b.launch()
            b.sync()
            st = b.stats()
            if k:
                ms.append(st.ms_filter)
            b.close()
        m = sum(ms) / len(ms)
        alg = st.in_bytes + st.stream_bytes
        print(f"{names[f]:9s} filter_ms {m:.3f} alg_bytes {alg} gbps {alg / m / 1e6:.1f} "
              f"frac {alg / m / 1e6 / 8000:.3f} deflate_ms {st.ms_deflate:.3f} out {st.deflate_out_bytes}",
              flush=True)
