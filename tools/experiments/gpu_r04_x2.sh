# cfg-3 shard with 1/2/3 calls in flight (every stream warmed before timing); the K2 floor probe;
# K2 with non-temporal bucket stores.
set -o pipefail
OUT=gpurun_out/r04x2; mkdir -p $OUT
for inf in 1 2 3 1 2 3; do
  echo -n "inflight $inf " >> $OUT/cfg3_inflight.txt
  timeout -k 10 120 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf 2>&1 | grep "batch n" >> $OUT/cfg3_inflight.txt || exit 1
done
timeout -k 10 120 tools/experiments/k2_stream_probe > $OUT/k2_stream_probe.txt 2>&1 || exit 1
bash tools/experiments/gpu_k2_libs.sh r04x2 tree=tree ntst=opendht_amd/ab/k2_ntst.so ntst_p4=opendht_amd/ab/k2_ntst_p4u4.so > /dev/null || exit 1
echo ok
