"""Served-path tuning: pbx_serve_bench at several caller counts x coalescer depths x batch
caps (PBX_COALESCE_DEPTH / PBX_MAX_BATCH are read when a context is created).
usage: serve_sweep.py DEPTHS [MAXBATCHES [THREADS]]  (comma lists)"""
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
maxb = [int(m) for m in (sys.argv[2] if len(sys.argv) > 2 else "65536").split(",")]
threads = tuple(int(t) for t in (sys.argv[3] if len(sys.argv) > 3 else "8,32,128,512").split(","))
for depth in [int(d) for d in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(",")]:
    for mb in maxb:
        os.environ["PBX_COALESCE_DEPTH"] = str(depth)
        os.environ["PBX_MAX_BATCH"] = str(mb)
        with pbx.PixelsService(device=0) as svc:
            svc.register_plane(1, 0, 0, 0, pbx.UINT16, 32768, 32768, generator="noise", seed=0)
            key = f"depth_{depth}_maxbatch_{mb}"
            out[key] = bench.serve_lines(svc, 1, threads=threads)
        print(json.dumps({key: out[key]}), flush=True)
