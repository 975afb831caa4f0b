# round 6: prefix / shard shapes with sorted sub-partitions (k_f2_direct) vs the unsorted default
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2; do
for b in tree v_sort; do
  e=""; [ $b != tree ] && e="DHTGPU_LIB=opendht_amd/ab/$b.so"
  timeout -k 10 300 env $e X=1 python tools/batch_probe.py --reps 20 --inflight 2 --cfg3 prefix > $OUT/prefix_${b}_$i.log 2>&1 || { tail -5 $OUT/prefix_${b}_$i.log; exit 1; }
  echo "prefix $b $i: $(grep -h 'ms/call' $OUT/prefix_${b}_$i.log) | $(grep -h phases $OUT/prefix_${b}_$i.log)"
  timeout -k 10 300 env $e X=1 python tools/batch_probe.py --reps 20 --inflight 2 --n 134217728 --q 131072 > $OUT/shard_${b}_$i.log 2>&1 || { tail -5 $OUT/shard_${b}_$i.log; exit 1; }
  echo "shard $b $i: $(grep -h 'ms/call' $OUT/shard_${b}_$i.log) | $(grep -h phases $OUT/shard_${b}_$i.log)"
done
done
