# round 6: F1 two-pass + F3 record-form experiments.  usage: bash tools/experiments/gpu_r06_rec.sh tag
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "record or merge or cfg3 or shard or sub_handles or fuzz or tie" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in tree h8; do
  e=""; [ $lib != tree ] && e="DHTGPU_LIB=opendht_amd/ab/$lib.so"
  timeout -k 10 300 env $e X=1 python tools/experiments/rec_vs_idx.py broadcast > $OUT/rec_$lib.log 2>&1 || { tail -5 $OUT/rec_$lib.log; exit 1; }
  echo "$lib: $(tail -2 $OUT/rec_$lib.log | tr '\n' ' ')"
done
for b in tree h8; do
  e=""; [ $b != tree ] && e="DHTGPU_LIB=opendht_amd/ab/$b.so"
  for r in broadcast prefix; do
    timeout -k 10 300 env $e X=1 python tools/batch_probe.py --reps 20 --inflight 2 --cfg3 $r > $OUT/${r}_$b.log 2>&1 || { tail -5 $OUT/${r}_$b.log; exit 1; }
    echo "$r $b: $(grep -h 'ms/call' $OUT/${r}_$b.log) | $(grep -h phases $OUT/${r}_$b.log)"
  done
done
