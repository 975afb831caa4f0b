# Non-temporal stream loads (DHT_STREAM_NT: F2 / S1 rings; DHT_K2_NT: K2 planes) and K2 without
# its global histogram atomics (DHT_K2_NOHIST, results wrong), against the in-tree build.
set -o pipefail
OUT=gpurun_out/ntab; mkdir -p $OUT
bash tools/experiments/gpu_k2_libs.sh ntab tree=tree nohist=opendht_amd/ab/k2nohist.so k2nt=opendht_amd/ab/k2nt.so || exit 1
for i in 1 2; do
  for nv in tree=tree streamnt=opendht_amd/ab/streamnt.so; do
    p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
    echo -n "${nv%%=*} "; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 1 8 2>/dev/null | tr '\n' ' '; echo
  done
done | tee $OUT/ks.txt
bash tools/experiments/gpu_ab_libs.sh ntab2 none tree=tree streamnt=opendht_amd/ab/streamnt.so
