"""configs[4] workload alone (the bench's c5_mixed_16384_requests line): the 16,384-request
mixed stream over uint8 / int32 / float32 16384^2 planes, in batches of 2048, pipelined two
deep as bench.py runs it.  Prints tiles/s per pass, then (one kernel stream) each batch's
stage times summed over the pass: k_extract (raw / TIFF), the PNG row kernels, the deflate
chain.  Used under rocprofv3 --kernel-trace (profiles/r06*/c5_*).

    python scripts/c5_pass.py [passes]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
sys.path.insert(0, ROOT)
import pbx  # noqa: E402
import bench  # noqa: E402

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 3
svc = pbx.PixelsService(device=0)
for k, pt in enumerate((pbx.UINT8, pbx.INT32, pbx.FLOAT)):
    svc.register_plane(10 + k, 0, 0, 0, pt, bench.C5_SIDE, bench.C5_SIDE, generator="noise")
reqs = bench.c5_stream()
chunks = [pbx.make_reqs(reqs[j:j + 2048]) for j in range(0, len(reqs), 2048)]


def one_pass():
    stats, prev = [], None
    for r in chunks + [None]:
        b = None
        if r is not None:
            b = pbx.Batch(svc, reqs=r)
            b.launch()
        if prev is not None:
            prev.sync()
            stats.append(prev.stats())
            prev.close()
        prev = b
    return stats


one_pass()
for p in range(passes):
    t0 = time.perf_counter()
    st = one_pass()
    dt = time.perf_counter() - t0
    ok = sum(s.ok_tiles for s in st)
    print(f"pass {p}: {dt * 1e3:.2f} ms, {ok / dt:.1f} tiles/s ({ok} ok)", flush=True)
svc.set_kernel_streams(1, 0)
st = one_pass()
tot = {f: sum(getattr(s, f) for s in st) for f in ("ms_extract", "ms_filter", "ms_deflate", "ms_assemble",
                                                   "ms_total", "in_bytes", "stream_bytes", "out_bytes")}
raw_tif_in = sum(s.in_bytes for s in st)  # (all tiles; PNG tiles' bytes are in stream_bytes too)
print("serial pass:", {k: round(v, 3) if isinstance(v, float) else v for k, v in tot.items()}, flush=True)
svc.close()
