"""Print the steady-state K6 timeline of a pipelined kernel trace: every dispatch of a window
of successive calls with its queue, start and end relative to the window (µs), so that the
order the dispatcher gave F2 / F3 / F4 of the two streams can be read off.
usage: kt_timeline.py TRACE_DIR [first_call] [ncalls]"""
import csv
import glob
import re
import sys

d = sys.argv[1]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 300
nc = int(sys.argv[3]) if len(sys.argv) > 3 else 6
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_f\d\w*)", r["Kernel_Name"])
        if m:
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1), q, int(r.get("Correlation_Id", 0) or 0)))
rows.sort(key=lambda x: x[4] or x[0])
f2 = [i for i, r in enumerate(rows) if r[2].startswith("k_f2")]
lo = f2[first] - 1
hi = f2[first + nc]
win = sorted(rows[lo:hi], key=lambda x: x[0])
t0 = win[0][0]
for s, e, k, q, c in win:
    print(f"{k:14s} q{q:>3s} start {(s - t0) / 1e3:8.2f} end {(e - t0) / 1e3:8.2f} dur {(e - s) / 1e3:6.2f}")
