# Round 5, pass q: the cfg-3 shard (2^27 ids, 131,072 targets) with w0 ties answered inline in F3
# (tieinline2.so) against the in-tree build (ties deferred to F4), one and two calls in flight.
set -o pipefail
OUT=gpurun_out/r05q; mkdir -p $OUT
for i in 1 2; do
  for lib in "" opendht_amd/ab/tieinline2.so; do
    for inf in 1 2; do
      echo "lib=${lib:-intree} inflight=$inf" >> $OUT/cfg3.txt
      DHTGPU_LIB=$lib timeout -k 10 200 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf >> $OUT/cfg3.txt 2>&1 || { tail -20 $OUT/cfg3.txt; exit 1; }
    done
  done
done
grep -E "lib=|phases|ms/call" $OUT/cfg3.txt
