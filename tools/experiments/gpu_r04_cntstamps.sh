# F2 phase stamps, A (opendht_amd/ab/prev.so: ranking flush) vs B (in-tree: counted flush), cfg 2 and the cfg-3 shard
set -o pipefail
OUT=gpurun_out/r04cnts; mkdir -p $OUT
for L in A B; do
  E=$([ $L = A ] && echo DHTGPU_LIB=opendht_amd/ab/prev.so || echo B=1)
  timeout -k 10 120 env DHTGPU_DBG=256 $E python tools/batch_probe.py --reps 3 > $OUT/cfg2_$L.log 2>&1 &&
  timeout -k 10 120 env DHTGPU_DBG=256 $E python tools/batch_probe.py --reps 3 --n 134217728 --q 131072 > $OUT/cfg3_$L.log 2>&1 || exit 1
done
for f in $OUT/*.log; do echo "== $f"; grep -E "F2 (stream|flush|end)" $f | tail -5; done
