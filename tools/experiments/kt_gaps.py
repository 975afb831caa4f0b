"""Summarise a rocprofv3 kernel trace: per-kernel mean duration, and the mean gap between the
end of one K6 kernel and the start of the next (one call = F1 F2 F3 F4).  usage: kt_gaps.py DIR"""
import collections
import csv
import glob
import re
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:30]))
rows.sort()
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for i, (s, e, k) in enumerate(rows):
    dur[k].append((e - s) / 1e3)
    if i and rows[i - 1][2].startswith("k_f") and k.startswith("k_f"):
        gap[rows[i - 1][2] + "->" + k].append((s - rows[i - 1][1]) / 1e3)
for k, v in sorted(dur.items()):
    v = sorted(v)
    print(f"{k:24s} n={len(v):4d} mean {sum(v) / len(v):8.2f} us  median {v[len(v) // 2]:8.2f} us")
for k, v in sorted(gap.items()):
    v = sorted(v)
    print(f"gap {k:36s} n={len(v):4d} median {v[len(v) // 2]:6.2f} us")
