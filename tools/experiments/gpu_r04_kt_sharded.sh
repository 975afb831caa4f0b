# kernel trace of the world-of-one collective path (K6 record mode + RCCL exchange + K3)
set -o pipefail
OUT=gpurun_out/${1:-r04ktsh}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --sharded --steps 20 --warmup 5 --no-cpu --no-extra --no-scan --inflight 1 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us avg", r["Percentage"])
PY
