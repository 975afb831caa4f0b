# Round 5, pass v: sub-partition handles -- the sub-partition suites and the new handle tests,
# then the cfg-3 shard with and without handles (two in flight), and F3's PMC bytes with handles.
set -o pipefail
OUT=gpurun_out/r05v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_fuzz.py -k "handles or sub or cfg3 or record" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for h in "" --handles; do
    echo -n "cfg3 ${h:-indices} "; timeout -k 10 200 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight 2 $h 2>&1 | grep -E "ms/call|phases" | tr '\n' ' ' || exit 1; echo
  done
done | tee $OUT/cfg3_handles.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/h_fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 --handles > $OUT/h_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/h_write -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 --handles > $OUT/h_write.log 2>&1 &&
cp profiles/r05/pmc_traffic.json $OUT/pmc_traffic.json &&
python3 tools/pmc_traffic.py $OUT/h_fetch $OUT/h_write $OUT/pmc_traffic.json "cfg3shard:134217728x131072x8:handles" > $OUT/h_pmc.txt || exit 1
grep -A3 k_f3_answer $OUT/h_pmc.txt | head -5
echo all-ok
