"""Pipelined K6 timeline from a rocprofv3 kernel trace: how much of each kernel's time
overlaps a kernel of another in-flight batch (F2 vs F3 etc.), and a sample of the
timeline.  usage: kt_overlap.py DIR"""
import collections
import csv
import glob
import re
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_f\d\w*)", r["Kernel_Name"])
        if m:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1)))
rows.sort()
rows = rows[len(rows) // 4:]   # skip warmup / setup
ov = collections.defaultdict(float)
tot = collections.defaultdict(float)
for i, (s, e, k) in enumerate(rows):
    tot[k] += e - s
    for j in range(max(0, i - 12), min(len(rows), i + 12)):
        if j == i:
            continue
        s2, e2, k2 = rows[j]
        x = min(e, e2) - max(s, s2)
        if x > 0:
            ov[(k, k2)] += x
for (k, k2), x in sorted(ov.items()):
    print(f"{k:16s} overlapped by {k2:16s} {100 * x / tot[k]:5.1f} % of its time")
busy, cur_s, cur_e = 0, None, None
for s, e, _ in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = rows[-1][1] - rows[0][0]
print(f"span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / span:.1f} %), "
      f"{sum(1 for r in rows if r[2].startswith('k_f2'))} F2 launches")
t0 = rows[0][0]
for s, e, k in rows[:24]:
    print(f"  {k:16s} {(s - t0) / 1e3:8.2f} .. {(e - t0) / 1e3:8.2f}  ({(e - s) / 1e3:6.2f})")
