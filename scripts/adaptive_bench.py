"""Runs bench.py's adaptive-filter line alone (1 GPU), prints its JSON."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

pbx = bench.pbx
torch.cuda.set_device(0)
with pbx.PixelsService(device=0) as svc:
    print(json.dumps(bench.adaptive_filter_line(svc, 0, 1, lambda: None, bench.GRID * bench.TILE)), flush=True)
