"""Sub-batch probe (lever 1): does the deflate chain get faster when the
filtered stream k_lz77 writes and k_encode reads back stays inside the 256 MiB Infinity Cache?

The headline's 4096 tiles (512x512 uint16 G_NOISE -> PNG) are cut into batches of N tiles
(stream bytes per batch = N x 525 KB: 4096 -> 2.15 GB, 256 -> 134 MB), run back to back on ONE
kernel stream; per step the kernels' HIP-event times are summed over the batches.

    python scripts/subbatch_probe.py [steps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import pbx  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
sizes = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [4096, 1024, 512, 256, 128]
svc = pbx.PixelsService(device=0)
side = 32768
svc.register_plane(1, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0)
grid = [pbx.TileCtx(1, 0, 0, 0, (i % 64) * 512, (i // 64) * 512, 512, 512, format="png")
        for i in range(4096)]
svc.set_kernel_streams(int(os.environ.get("PROBE_KSTREAMS", "1")), 1 if os.environ.get("PROBE_KSTREAMS") else 0)
out = {}
for n in sizes:
    reqs = [pbx.make_reqs(grid[j:j + n]) for j in range(0, 4096, n)]

    def one_step(record):
        q, acc = [], {"lz77": 0.0, "huff": 0.0, "encode": 0.0, "total": 0.0}
        for r in reqs:
            b = pbx.Batch(svc, reqs=r)
            b.launch()
            q.append(b)
            if len(q) >= 3:
                f = q.pop(0)
                f.sync()
                if record:
                    s = f.stats()
                    acc["lz77"] += s.ms_lz77
                    acc["huff"] += s.ms_huff
                    acc["encode"] += s.ms_encode
                    acc["total"] += s.ms_total
                f.close()
        for f in q:
            f.sync()
            if record:
                s = f.stats()
                acc["lz77"] += s.ms_lz77
                acc["huff"] += s.ms_huff
                acc["encode"] += s.ms_encode
                acc["total"] += s.ms_total
            f.close()
        return acc

    one_step(False)
    one_step(False)
    svc.synchronize()
    t0 = time.perf_counter()
    accs = [one_step(True) for _ in range(steps)]
    svc.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    mean = {k: round(sum(a[k] for a in accs) / steps, 3) for k in accs[0]}
    out[n] = {"wall_ms_per_4096": round(wall, 3), "kernel_ms_per_4096": mean,
              "tiles_per_s": round(4096 / wall * 1e3, 1)}
    print(json.dumps({n: out[n]}), flush=True)
    svc.release_cached()
print(json.dumps(out))
