# One PMC pass: LDS stall counters per kernel over the profiling workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS -d gpurun_out/pmcl -o run --output-format csv -- python3 scripts/prof_workload.py noise 2 > gpurun_out/pmcl.log 2>&1 || { echo pmcl FAIL; tail -20 gpurun_out/pmcl.log; exit 1; }
python3 - <<'PY'
import csv, glob
from collections import defaultdict
f = glob.glob("gpurun_out/pmcl/*counter_collection.csv")[0]
per = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    per[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, cs in per.items():
    d = len(n[k]); w = cs.get("SQ_WAVES", 1) or 1
    print(k, " ".join(f"{c}={v/d:.4g} ({v/w:.1f}/wave)" for c, v in sorted(cs.items())))
PY
