# round 6: the driver-shaped bench (headline cfg 2 only) with two builds, alternating
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for i in 1 2; do
for b in "$@"; do
  e=""; [ $b != tree ] && e="DHTGPU_LIB=opendht_amd/ab/$b.so"
  timeout -k 10 200 env $e X=1 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > $OUT/b20_${b}_$i.json 2> $OUT/b20_${b}_$i.err || { tail -5 $OUT/b20_${b}_$i.err; exit 1; }
  timeout -k 10 200 env $e X=1 python bench.py --steps 1000 --warmup 100 --no-cpu --no-extra > $OUT/b1000_${b}_$i.json 2> $OUT/b1000_${b}_$i.err || { tail -5 $OUT/b1000_${b}_$i.err; exit 1; }
  python3 - $OUT/b20_${b}_$i.json $OUT/b1000_${b}_$i.json $b <<'PY'
import json, sys
a = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "20 steps %.2f us" % (a["ms_per_step"] * 1e3), "lat %.1f" % (a["latency_ms_per_batch"] * 1e3), "| 1000 steps %.2f us" % (c["ms_per_step"] * 1e3), "verified", a.get("verified_exact"))
PY
done
done
