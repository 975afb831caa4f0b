# same-box A/B of the cfg-3 shard (2^27 ids x 131,072 targets, plain set -> 8 sorted sub-partitions)
# and the per-rank shapes: in-tree build vs a baseline build.  usage: bash ... tag base.so
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2; do
  for b in tree base; do
    lib=""; [ $b = base ] && lib="DHTGPU_LIB=$2"
    timeout -k 10 300 env $lib X=1 python tools/batch_probe.py --reps 20 --inflight 2 --n 134217728 --q 131072 > $OUT/shard_${b}_$i.log 2>&1 || { tail -5 $OUT/shard_${b}_$i.log; exit 1; }
    echo "shard $b $i: $(grep -h 'ms/call' $OUT/shard_${b}_$i.log) | $(grep -h phases $OUT/shard_${b}_$i.log)"
  done
done
for b in tree base; do
  lib=""; [ $b = base ] && lib="DHTGPU_LIB=$2"
  for r in broadcast prefix; do
    timeout -k 10 300 env $lib X=1 python tools/batch_probe.py --reps 20 --inflight 2 --cfg3 $r > $OUT/${r}_$b.log 2>&1 || { tail -5 $OUT/${r}_$b.log; exit 1; }
    echo "$r $b: $(grep -h 'ms/call' $OUT/${r}_$b.log) | $(grep -h phases $OUT/${r}_$b.log)"
  done
done
