"""Per-kernel SQ counter summary from rocprofv3 --pmc passes (run_counter_collection.csv in each
directory given): mean per dispatch of every counter, and derived figures -- VALU instructions
per SIMD-cycle (GRBM_GUI_ACTIVE / 8 = cycles per XCD; 4 SIMDs x 32 CUs per XCD), the fraction of
wave time spent waiting, LDS bank-conflict cycles per LDS instruction.
usage: python tools/pmc_sq_summary.py DIR [DIR ...] > summary.txt"""
import collections
import csv
import os
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k in sorted(acc):
    if not k.startswith("k_f") and not k.startswith("k_s") and not k.startswith("k_cl"):
        continue
    c = {n: v / max(1, len(disp[(k, n)])) for n, v in acc[k].items()}
    print(k)
    for n in sorted(c):
        print(f"  {n:24s} {c[n]:.4e}")
    g = c.get("GRBM_GUI_ACTIVE")
    if g and c.get("SQ_INSTS_VALU"):
        cyc = g / 8
        print(f"  -> VALU instr per SIMD-cycle {c['SQ_INSTS_VALU'] / (cyc * 1024):.4f} (1.0 = every SIMD issuing VALU every cycle)")
    if c.get("SQ_WAVE_CYCLES") and c.get("SQ_WAIT_ANY"):
        print(f"  -> waiting fraction of wave time {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
    if c.get("SQ_LDS_BANK_CONFLICT") and c.get("SQ_ACTIVE_INST_LDS"):
        print(f"  -> LDS bank-conflict cycles per active LDS cycle {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_ACTIVE_INST_LDS']:.3f}")
