"""Per-kernel instruction mix of a device assembly file (hipcc --save-temps): counts of VALU,
SALU, LDS, global/buffer memory, DPP and v_cndmask instructions in the kernel's text (static
counts, all paths), and the register / LDS footprint from the kernel descriptor.

    python scripts/isa_stats.py file.s [name-substring ...]"""
import re
import sys


def kernels(path):
    cur, out = None, {}
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;|$)", line)
        if m:
            cur = m.group(1)
            out[cur] = {"lines": []}
            continue
        if cur and line.startswith("\t.size\t" + cur):
            cur = None
            continue
        if cur:
            out[cur]["lines"].append(line.strip())
    # the per-function comment block after each kernel: "; NumVgprs: n", "; Occupancy: n", ...
    meta, last = {}, None
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;|$)", line)
        if m:
            last = m.group(1)
        m = re.match(r"^; (NumVgprs|NumSgprs|ScratchSize|Occupancy|LDSByteSize): (\d+)", line)
        if m and last:
            meta.setdefault(last, {})[m.group(1)] = int(m.group(2))
    return out, meta


def stats(lines):
    c = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "dpp": 0, "cndmask": 0, "branch": 0}
    for l in lines:
        if not l or l.startswith((";", ".")) or l.endswith(":"):
            continue
        op = l.split()[0]
        if op.startswith("v_"):
            c["valu"] += 1
            if "dpp" in l or "row_" in l or "wave_" in l:
                c["dpp"] += 1
            if op.startswith("v_cndmask"):
                c["cndmask"] += 1
        elif op.startswith("s_cbranch") or op.startswith("s_branch"):
            c["branch"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
    return c


if __name__ == "__main__":
    ks, meta = kernels(sys.argv[1])
    subs = sys.argv[2:]
    for k, v in ks.items():
        if subs and not any(s in k for s in subs):
            continue
        print(k[:90], stats(v["lines"]), meta.get(k, {}))
