"""The deflate chain on the bench's Poisson-like plane (adaptive_filter_line's: 32768^2 uint16,
lambda drifting 200..300) under filter None and the adaptive option, next to G_NOISE under
filter None: 4096 x 512^2 PNG tiles a batch, serial kernel stream, per-phase HIP-event ms and
output bytes.  Run under rocprofv3 --kernel-trace for the per-kernel split."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import pbx  # noqa: E402

side = 32768
yy, xx = np.mgrid[0:side:64, 0:side:64]
lam = 200.0 + 100.0 * (0.5 + 0.25 * np.sin(xx / 900.0) + 0.25 * np.cos(yy / 1300.0))
gen = torch.Generator(device="cuda").manual_seed(1234)
lam_t = torch.from_numpy(lam.astype(np.float32)).cuda().repeat_interleave(64, 0).repeat_interleave(64, 1)
pois = torch.poisson(lam_t, generator=gen).to(torch.int16).cpu().numpy().view(np.uint16)
del lam_t
for name, filt, data in (("noise/none", 0, None), ("poisson/none", 0, pois), ("poisson/adaptive", 5, pois)):
    with pbx.PixelsService(device=0, png_filter=filt) as svc:
        svc.set_kernel_streams(1, 0)
        if data is None:
            svc.register_plane(1, 0, 0, 0, pbx.UINT16, side, side, generator="noise")
        else:
            svc.register_plane(1, 0, 0, 0, pbx.UINT16, side, side, data=data, big_endian=False)
        ctxs = [pbx.TileCtx(1, 0, 0, 0, (i % 64) * 512, (i // 64) * 512, 512, 512, format="png")
                for i in range(4096)]
        reqs = pbx.make_reqs(ctxs)
        rows = []
        for k in range(4):
            b = pbx.Batch(svc, reqs=reqs)
            b.launch()
            b.sync()
            st = b.stats()
            if k:
                rows.append((st.ms_filter, st.ms_deflate, st.ms_assemble, st.ms_total))
            b.close()
        m = np.mean(np.array(rows), 0)
        print(f"{name:17s} filter {m[0]:.3f} deflate {m[1]:.3f} assemble {m[2]:.3f} total {m[3]:.3f} ms "
              f"out {st.deflate_out_bytes / 4096:.0f} B/tile segments {st.segments} blocks {st.blocks} "
              f"direct {st.direct_tiles}", flush=True)
