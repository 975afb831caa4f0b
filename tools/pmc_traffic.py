"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), per kernel.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json WORKLOAD
FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of wide
(16 B/lane) streaming reads (MI355X_MICROARCH.md, HBM section): it is doubled here.
WRITE_SIZE is taken as is.  Infinity-Cache hits are counted by these counters, so only a
workload that does not fit the 256 MiB L3 (or evicts it between calls) reads as HBM traffic.
Results are merged into OUT.json under workloads[WORKLOAD] (the key bench.py looks up)."""
import collections
import csv
import json
import os
import re
import sys


def per_kernel(d, counter):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        acc[(m.group(1) if m else r["Kernel_Name"][:40], r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = collections.defaultdict(list)
    for (k, _), v in acc.items():
        out[k].append(v * 1024.0)
    return {k: sum(v) / len(v) for k, v in out.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
res = {}
for k in sorted(set(fetch) | set(write)):
    f = 2.0 * fetch.get(k, 0.0)
    w = write.get(k, 0.0)
    res[k] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w}
try:
    doc = json.load(open(sys.argv[3]))
except (OSError, ValueError):
    doc = {}
doc["note"] = ("per-launch HBM-side bytes: 2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, averaged over "
               "the launches of each kernel; separate rocprofv3 --pmc passes on tools/batch_probe.py")
key = sys.argv[4]
if key.startswith("@"):   # the probe wrote the key (its shape is known only after its setup)
    key = open(key[1:]).read().strip()
doc.setdefault("workloads", {})[key] = res
json.dump(doc, open(sys.argv[3], "w"), indent=1)
print(key, json.dumps(res, indent=1))
