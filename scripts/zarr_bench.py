"""Row f2 alone: bench.py's Zarr decode line (for rocprofv3 kernel traces of k_zarr_*)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

with bench.pbx.PixelsService(device=0) as svc:
    print(json.dumps(bench.zarr_lines(svc, 0, 1)), flush=True)
