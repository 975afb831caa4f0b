# Round 5, pass h: the cfg-3 shard (2^27 ids, 131,072 targets) with F3's result-map reads left out
# (opendht_amd/ab/nomap.so, -DDHT_F3_NOMAP: sub-partition-local results, a measurement only)
# against the in-tree build, one and two calls in flight.   usage: bash tools/experiments/gpu_r05_h.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r05h}; mkdir -p $OUT
for i in 1 2; do
  for lib in "" opendht_amd/ab/nomap.so; do
    for inf in 1 2; do
      echo "lib=${lib:-intree} inflight=$inf" >> $OUT/cfg3_nomap.txt
      DHTGPU_LIB=$lib timeout -k 10 200 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf >> $OUT/cfg3_nomap.txt 2>&1 || { tail -20 $OUT/cfg3_nomap.txt; exit 1; }
    done
  done
done
grep -E "lib=|phases|ms/call" $OUT/cfg3_nomap.txt
echo all-ok
