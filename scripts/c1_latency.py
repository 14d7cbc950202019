"""configs[0]'s single-request latency, broken down: ONE 512x512 uint8 PNG
request (tile (0, 0) of a 4096^2 G_FAKE plane) at a time.

* the served path (pbx_get_tile through the coalescer; native caller loop, bench.serve_one):
  p50/p90/p99, and PBX_TIMELINE's per-stage split printed by the library at shutdown (queue ->
  launcher, plan, launch enqueue, kernels until the completer sees them done, D2H, caller
  wake-up);
* the batch spans of the served requests (pbx_result_spans: device first-to-last kernel, D2H);
* the same request through the synchronous batch API from this thread (plan / launch / sync /
  fetch host timings), no coalescer threads.

Usage: PBX_TIMELINE=1 python scripts/c1_latency.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import bench  # noqa: E402
import pbx  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
svc = pbx.PixelsService(device=0)
svc.register_plane(6, 0, 0, 0, pbx.UINT8, 4096, 4096, generator="fake", plane_no=0)
tc = pbx.TileCtx(6, 0, 0, 0, 0, 0, 512, 512, format="png")
print("served", bench.serve_one(svc, [tc], 1, reps, 200), flush=True)
sp = []
for _ in range(50):
    d = {}
    st, body = svc.get_tile(tc, spans=d)
    assert st == 0
    sp.append(d)
sp = sp[10:]
print("spans ms (median):", {k: round(sorted(x[k] for x in sp)[len(sp) // 2], 4)
                            for k in ("batch_ms", "d2h_ms", "write_image_ms", "create_metadata_ms")}, flush=True)
t = {"plan": [], "launch": [], "sync": [], "fetch": [], "total": []}
reqs = pbx.make_reqs([tc])
for i in range(300):
    t0 = time.perf_counter()
    b = pbx.Batch(svc, reqs=reqs)
    t1 = time.perf_counter()
    b.launch()
    t2 = time.perf_counter()
    b.sync()
    t3 = time.perf_counter()
    n = b.fetch_into_host()
    t4 = time.perf_counter()
    b.close()
    if i >= 50:
        for k, v in (("plan", t1 - t0), ("launch", t2 - t1), ("sync", t3 - t2), ("fetch", t4 - t3), ("total", t4 - t0)):
            t[k].append(v * 1e6)
print("batch api us (median):", {k: round(sorted(v)[len(v) // 2], 1) for k, v in t.items()}, flush=True)
svc.close()
