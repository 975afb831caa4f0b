# Sub-partitioned calls' result-map reads (gidx, one random 4-B read per result) non-temporal
# (-DDHT_MAP_NT) against the in-tree build, on the cfg-3 shard probe; sub-partition tests first.
set -o pipefail
OUT=gpurun_out/mapnt; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/mapnt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_scale.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3; do
  for nv in tree=tree mapnt=opendht_amd/ab/mapnt.so; do
    p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
    echo "${nv%%=*} $(timeout -k 10 200 env $lib X=1 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 2>/dev/null | grep -h 'phases\|ms/call' | tr '\n' ' ')" || exit 1
  done
done | tee $OUT/ab.txt
