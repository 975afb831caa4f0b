# Round 5, pass b: K2 builds A/B (deferred exact path, workgroups per CU, ids per lane), the
# per-rank K6 record-form timings at the N = 1/2/4/8 shard sizes, and a kernel trace of the
# world-of-one collective path.   usage: bash tools/experiments/gpu_r05_b.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r05b}; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/experiments/gpu_k2_libs.sh ${1:-r05b} prev=opendht_amd/ab/prev.so new=tree u3pc5=opendht_amd/ab/u3pc5.so \
  u2pc6=opendht_amd/ab/u2pc6.so u2pc7=opendht_amd/ab/u2pc7.so u2pc8=opendht_amd/ab/u2pc8.so || exit 1
for i in 1 2; do
  for nv in new=tree s1r2=opendht_amd/ab/s1r2.so s1r4=opendht_amd/ab/s1r4.so; do
    p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
    for ev in "" --evict; do
      echo "== ${nv%%=*} $ev"; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 1 8 32 64 --reps 10 $ev 2>/dev/null || exit 1
    done
  done
done | tee $OUT/ks_ab.txt
timeout -k 10 300 python tools/shard_probe.py > $OUT/shard_probe.json 2> $OUT/shard_probe.err || { tail -20 $OUT/shard_probe.err; exit 1; }
tail -1 $OUT/shard_probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_sharded -o run --output-format csv -- python3 bench.py --sharded --steps 20 --warmup 5 --no-cpu --no-extra --no-scan > $OUT/kt_sharded.log 2>&1 || exit 1
python3 - $OUT <<'PY'
import csv, glob, sys
o = sys.argv[1]
f = glob.glob(f"{o}/kt_sharded/**/*kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    print("kt_sharded", row["Name"].split("(")[0].replace("dhtgpu::(anonymous namespace)::", "")[:50], row["Calls"],
          round(float(row["AverageNs"]) / 1e3, 2), "us")
PY
echo all-ok
