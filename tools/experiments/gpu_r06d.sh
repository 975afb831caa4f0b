set -o pipefail
OUT=gpurun_out/r06d; mkdir -p $OUT
export DHTGPU_VERBOSE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 240 --timeout-method thread -m gpu -k "sibling" > $OUT/t_sib.log 2>&1 || { tail -30 $OUT/t_sib.log; exit 1; }
tail -1 $OUT/t_sib.log
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "cfg3 or subpartition or sub_handles or clustered or fuzz or tie_words or merge" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in broadcast prefix; do
  timeout -k 10 300 python tools/batch_probe.py --reps 20 --inflight 2 --cfg3 $r > $OUT/$r.log 2>&1 || { tail -5 $OUT/$r.log; exit 1; }
  echo "$r: $(grep -h 'ms/call' $OUT/$r.log) | $(grep -h phases $OUT/$r.log)"
done
if [ -n "$STAMPS" ]; then
  timeout -k 10 300 env DHTGPU_DBG=256 python tools/batch_probe.py --reps 2 --cfg3 prefix > $OUT/stamps_prefix.log 2>&1 || { tail -5 $OUT/stamps_prefix.log; exit 1; }
  grep -E "F2 " $OUT/stamps_prefix.log | tail -7
fi
