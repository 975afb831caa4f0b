"""Compare two pipelined kernel traces: per-kernel duration percentiles in the steady window
and the period between successive F2 starts.  usage: kt_pipe_cmp.py DIR_A DIR_B"""
import csv
import glob
import re
import sys

import numpy as np


def load(d):
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_f\d\w*)", r["Kernel_Name"])
            if m:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1)))
    rows.sort()
    n = len(rows)
    return rows[n // 3: n - n // 10]


for d in sys.argv[1:]:
    rows = load(d)
    print(d)
    for k in sorted({r[2] for r in rows}):
        dur = np.array([(e - s) / 1e3 for s, e, kk in rows if kk == k])
        print(f"  {k:14s} n={len(dur):4d} p10 {np.percentile(dur, 10):6.2f} p50 {np.percentile(dur, 50):6.2f} p90 {np.percentile(dur, 90):6.2f}")
    f2s = np.array([s for s, e, kk in rows if kk.startswith("k_f2")]) / 1e3
    print(f"  F2 start-to-start p50 {np.median(np.diff(f2s)):.2f} us, mean {np.mean(np.diff(f2s)):.2f}")
    # gaps: F3 start - F2 end of the same batch (stream order) approximated by the next F3 after each F2 end
    f2e = [e for s, e, kk in rows if kk.startswith("k_f2")]
    f3s = sorted(s for s, e, kk in rows if kk.startswith("k_f3"))
    gaps = []
    for e in f2e:
        nxt = [s for s in f3s if s >= e]
        if nxt:
            gaps.append((nxt[0] - e) / 1e3)
    print(f"  F2 end -> next F3 start p50 {np.median(gaps):.2f} us")
