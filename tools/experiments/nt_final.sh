# Non-temporal stream loads in production (S1 always; F2 for sub-partitioned sets past 192 MB of
# w0 planes): GPU suite, then the in-tree build against HEAD's on the KS probe, cfg 2 and cfg 3.
set -o pipefail
OUT=gpurun_out/ntfin; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for i in 1 2; do
  for nv in head=opendht_amd/ab/head.so tree=tree; do
    p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
    echo -n "${nv%%=*} "; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 1 8 64 2>/dev/null | tr '\n' ' '; echo
  done
done | tee $OUT/ks.txt
bash tools/experiments/gpu_ab_libs.sh ntfin2 none head=opendht_amd/ab/head.so tree=tree
