"""Summarise a gpu_cycle.sh run: kernel stats + derived VALU issue metrics for k_scan."""
import csv, collections, sys, os
d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_scan"
pairs = float(sys.argv[3]) if len(sys.argv) > 3 else 65536 * 2**24
for r in csv.DictReader(open(os.path.join(d, "kt", "run_kernel_stats.csv"))):
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]} avg_ms={float(r["AverageNs"])/1e6:.3f} pct={r["Percentage"]}')
agg = collections.defaultdict(float)
dur = 0
for f in ("pmc1", "pmc2"):
    p = os.path.join(d, f, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"  {k:24s} {v:.4e}")
if agg.get("GRBM_GUI_ACTIVE") and agg.get("SQ_INSTS_VALU"):
    cyc = agg["GRBM_GUI_ACTIVE"] / 8
    print(f"  cycles/XCD={cyc:.4e}  VALU instr/cycle/SIMD={agg['SQ_INSTS_VALU']/1024/cyc:.4f} (peak 0.25)"
          f"  VALU/pair={agg['SQ_INSTS_VALU']*64/pairs:.4f}  SALU/VALU={agg['SQ_INSTS_SALU']/agg['SQ_INSTS_VALU']:.3f}")
