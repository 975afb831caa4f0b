# round 6: cfg 2 through sorted sub-partitions (v_cfg2s) vs the one-set K6, 2 and 3 in flight
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for b in tree v_cfg2s; do
  e=""; [ $b != tree ] && e="DHTGPU_LIB=opendht_amd/ab/$b.so"
  for i in 2 3; do
    timeout -k 10 200 env $e X=1 python tools/batch_probe.py --reps 200 --inflight $i > $OUT/cfg2_${b}_$i.log 2>&1 || { tail -5 $OUT/cfg2_${b}_$i.log; exit 1; }
    echo "cfg2 $b inflight $i: $(grep -h ms/call $OUT/cfg2_${b}_$i.log | sed 's/batch //') | $(grep -h phases $OUT/cfg2_${b}_$i.log | cut -c1-70)"
  done
done
