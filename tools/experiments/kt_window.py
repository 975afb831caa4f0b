"""Per-kernel mean duration of the K6 calls [first, first + count) in a rocprofv3 kernel trace
(each K6 kernel's dispatches in start order: dispatch j of k_f2_filter belongs to call j).
bench.py --steps S --warmup W issues W warmup calls, S timed calls (two in flight), then
max(3, min(S, 20)) serial calls timed by events (the roofline's kernels_ms): so
`kt_window.py DIR W S` summarises the timed window and `kt_window.py DIR W+S R` the serial one.
usage: kt_window.py DIR FIRST COUNT"""
import collections
import csv
import glob
import re
import sys

d, first, count = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = collections.defaultdict(list)
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_f[1-4]\w*)", r["Kernel_Name"])
        if m:
            rows[m.group(1)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for k in sorted(rows):
    v = sorted(rows[k])[first:first + count]
    if v:
        ds = [(e - s) / 1e3 for s, e in v]
        print(f"{k:16s} calls {first}..{first + len(v) - 1}: mean {sum(ds) / len(ds):7.2f} us  "
              f"min {min(ds):7.2f}  max {max(ds):7.2f}")
