# Round 5, pass x: kernel trace of the world-of-one collective path at HEAD (K6 record form, the
# RCCL all-gather, K3), and of the cfg-3 shard with sub-partition handles.
set -o pipefail
OUT=gpurun_out/r05x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_sharded -o run --output-format csv -- python3 bench.py --sharded --steps 20 --warmup 5 --no-cpu --no-extra --no-scan > $OUT/kt_sharded.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg3_handles -o run --output-format csv -- python3 tools/batch_probe.py --reps 20 --n 134217728 --q 131072 --handles > $OUT/kt_cfg3_handles.log 2>&1 || exit 1
python3 - $OUT <<'PY'
import csv, glob, re, sys
o = sys.argv[1]
for k in ("kt_sharded", "kt_cfg3_handles"):
    f = glob.glob(f"{o}/{k}/**/*kernel_stats.csv", recursive=True)[0]
    for row in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+|__amd\w+|ncclDevKernel\w*|\w*Kernel\w*)", row["Name"])
        print(k, m.group(1) if m else row["Name"][:40], row["Calls"], round(float(row["AverageNs"]) / 1e3, 2), "us")
PY
echo all-ok
