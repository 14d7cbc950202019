"""One line of a bench.py JSON: value, deflate chain ms, k_lz77 / k_encode ms, serial pass rate."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(d["value"], d["deflate_chain_ms"], k["k_lz77"]["ms"], k["k_encode"]["ms"],
      d["kernel_streams"]["serial_pass_tiles_per_s"])
