# Round 5, pass u: tie slots by wave ballot (one LDS atomic per wave) instead of one atomic +
# shuffle per group.  cfg 2: inline (tree) / per-group hand-off (deferall) / ballot hand-off
# (deferball); the cfg-3 shard: ballot (tree) / per-group (pergroup).  Parity of the ballot
# builds first.
set -o pipefail
OUT=gpurun_out/r05u; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/deferball.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "batch or fuzz or record or cfg2 or clustered or fallback or w0" > $OUT/tests_deferball.log 2>&1 || { tail -30 $OUT/tests_deferball.log; exit 1; }
tail -1 $OUT/tests_deferball.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "cfg3 or subs or sub_part or 2p27 or records" > $OUT/tests_subs.log 2>&1 || { tail -30 $OUT/tests_subs.log; exit 1; }
tail -1 $OUT/tests_subs.log
for i in 1 2; do
  for v in tree deferall deferball; do
    lib=""; [ $v != tree ] && lib=opendht_amd/ab/$v.so
    echo -n "cfg2 $v "; DHTGPU_LIB=$lib timeout -k 10 120 python tools/batch_probe.py --reps 20 2>&1 | grep "phases ms" || exit 1
  done
  for v in tree pergroup; do
    lib=""; [ $v != tree ] && lib=opendht_amd/ab/$v.so
    echo -n "cfg3 $v "; DHTGPU_LIB=$lib timeout -k 10 200 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight 2 2>&1 | grep -E "ms/call|phases" | tr '\n' ' ' || exit 1; echo
  done
done | tee $OUT/ballot.txt
