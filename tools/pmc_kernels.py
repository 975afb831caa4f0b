"""Per-kernel averages of rocprofv3 counter passes: python pmc_kernels.py DIR pass1 [pass2 ...]
(sums a counter over a dispatch's rows, then averages over dispatches of the kernel)."""
import collections
import csv
import os
import re
import sys

d = sys.argv[1]
per = collections.defaultdict(float)          # (kernel, dispatch, counter) -> sum
for f in sys.argv[2:]:
    for r in csv.DictReader(open(os.path.join(d, f, "run_counter_collection.csv"))):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        kn = m.group(1) if m else r["Kernel_Name"][:40]
        per[(kn, f + r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
agg = collections.defaultdict(list)
for (kn, _, c), v in per.items():
    agg[(kn, c)].append(v)
kerns = sorted({k for k, _ in agg})
for kn in kerns:
    print(kn)
    for (k2, c), vs in sorted(agg.items()):
        if k2 == kn:
            print(f"   {c:24s} {sum(vs) / len(vs):.4e}   (n={len(vs)})")
