#!/usr/bin/env python3
"""Per-variant, per-layer median kernel times from a gemm8p_ab.py kernel trace: argv[1] = the
kernel_trace.csv; layers = the phase-interleaved dispatches of one launch in order."""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = [r for r in rows if "gemm8" in r["Kernel_Name"] or "gemm_k64p" in r["Kernel_Name"]]
out = defaultdict(lambda: defaultdict(list))
i = 0
while i < len(seq):
    name = seq[i]["Kernel_Name"]
    m = re.search(r"(gemm8p?_kernel|gemm_k64p_kernel)(<[^>]*>)?", name)
    key = m.group(1) + (m.group(2) or "")
    j = i
    layer = 0
    while j < len(seq) and seq[j]["Kernel_Name"] == name and layer < int(sys.argv[2] if len(sys.argv) > 2 else 3):
        out[key][layer].append((int(seq[j]["End_Timestamp"]) - int(seq[j]["Start_Timestamp"])) / 1e3)
        j += 1
        layer += 1
    i = j
print(json.dumps({k: {l: {"median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1), "n": len(v)}
                      for l, v in d.items()} for k, d in out.items()}, indent=1))
