"""Summarise rocprofv3 PMC passes (gpurun_out/pmc1..4) per kernel: mean counter values per
dispatch, per-wave instruction counts, and FETCH/WRITE bytes (FETCH_SIZE doubled for gfx950
wide streaming reads, MI355X_MICROARCH.md HBM section; sizes are in KB)."""
import csv
import glob
import os
import sys
from collections import defaultdict

import json

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
traffic_out = sys.argv[2] if len(sys.argv) > 2 else None
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(base, "pmc[1-9]", "*counter_collection.csv"))):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        k = k.split("<")[0]
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        per[(k, r["Dispatch_Id"])]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            vals[k][c].append(v)
for k, cs in sorted(vals.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    waves = m.get("SQ_WAVES", 0)
    line = [f"{k}: dur {m['_dur'] / 1e6:.3f} ms"]
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
              "SQ_BUSY_CYCLES", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_ANY",
              "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
              "SQ_INST_CYCLES_SALU"):
        if c in m:
            per_wave = f" ({m[c] / waves:.0f}/wave)" if waves and c != "SQ_WAVES" else ""
            line.append(f"{c} {m[c]:.4g}{per_wave}")
    if "FETCH_SIZE" in m:
        line.append(f"FETCH_SIZE x2 {2 * m['FETCH_SIZE'] * 1024 / 1e9:.3f} GB")
    if "WRITE_SIZE" in m:
        line.append(f"WRITE_SIZE {m['WRITE_SIZE'] * 1024 / 1e9:.3f} GB")
    print("\n   ".join(line))

if traffic_out:
    # HBM bytes per launch for bench.py's roofline "traffic" (FETCH_SIZE x2, WRITE_SIZE; KB units)
    t = {"workload": "scripts/prof_workload.py noise: 4096 x 512x512 uint16 G_NOISE tiles -> PNG",
         "rule": "fetch = 2 x FETCH_SIZE (gfx950 wide streaming reads), write = WRITE_SIZE; "
                 "mean per dispatch, separate rocprofv3 --pmc passes",
         "kernels": {}}
    for k, cs in sorted(vals.items()):
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
            t["kernels"][k.replace("pbx::", "")] = {"fetch_bytes": int(2 * f * 1024),
                                                     "write_bytes": int(w * 1024)}
    with open(traffic_out, "w") as fo:
        json.dump(t, fo, indent=1)
