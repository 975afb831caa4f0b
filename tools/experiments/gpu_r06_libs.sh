# same-box A/B of several builds on the cfg-3 per-rank shapes + the shard.
# usage: bash tools/experiments/gpu_r06_libs.sh tag lib1 lib2 ...   (tree = the in-tree build; others: opendht_amd/ab/<name>.so)
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for i in 1 2; do
for b in "$@"; do
  e=""; [ $b != tree ] && e="DHTGPU_LIB=opendht_amd/ab/$b.so"
  for r in prefix broadcast; do
    timeout -k 10 300 env $e X=1 python tools/batch_probe.py --reps 20 --inflight 2 --cfg3 $r > $OUT/${r}_${b}_$i.log 2>&1 || { tail -5 $OUT/${r}_${b}_$i.log; exit 1; }
    echo "$r $b $i: $(grep -h 'ms/call' $OUT/${r}_${b}_$i.log | sed 's/batch //') | $(grep -h phases $OUT/${r}_${b}_$i.log | cut -c1-60)"
  done
  timeout -k 10 300 env $e X=1 python tools/batch_probe.py --reps 20 --inflight 2 --n 134217728 --q 131072 > $OUT/shard_${b}_$i.log 2>&1 || { tail -5 $OUT/shard_${b}_$i.log; exit 1; }
  echo "shard $b $i: $(grep -h 'ms/call' $OUT/shard_${b}_$i.log | sed 's/batch //') | $(grep -h phases $OUT/shard_${b}_$i.log | cut -c1-60)"
done
done
