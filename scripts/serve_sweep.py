"""Served-path tuning: pbx_serve_bench at several caller counts x coalescer depths
(PBX_COALESCE_DEPTH is read when a context is created)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
import torch  # noqa: F401,E402
import bench  # noqa: E402
import pbx  # noqa: E402

out = {}
for depth in [int(d) for d in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(",")]:
    os.environ["PBX_COALESCE_DEPTH"] = str(depth)
    with pbx.PixelsService(device=0) as svc:
        svc.register_plane(1, 0, 0, 0, pbx.UINT16, 32768, 32768, generator="noise", seed=0)
        out[f"depth_{depth}"] = bench.serve_lines(svc, 1, threads=(8, 32, 128, 512))
    print(json.dumps({f"depth_{depth}": out[f"depth_{depth}"]}), flush=True)
