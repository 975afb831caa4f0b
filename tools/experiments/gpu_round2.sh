# Round-2 evidence on the GPU box: the GPU parity suite, PMC HBM traffic (separate FETCH_SIZE /
# WRITE_SIZE passes of tools/batch_probe.py: cfg 2 warm, cfg 2 with the Infinity Cache evicted,
# the 2^27-id cfg-3 shard), the default bench line (it reads that traffic file) and a
# rocprofv3 kernel trace + stats of the driver's bench command.
# usage: bash tools/gpu_round2.sh <out-tag> [skip-tests]
set -o pipefail
TAG=${1:-round}; OUT=gpurun_out/$TAG; mkdir -p $OUT profiles/r02
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
pmc() {  # name, workload key, probe args
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/$1_fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 $3 > $OUT/$1_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/$1_write -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 $3 > $OUT/$1_write.log 2>&1 &&
  python3 tools/pmc_traffic.py $OUT/$1_fetch $OUT/$1_write $OUT/pmc_traffic.json "$2" > $OUT/$1_pmc.txt && cp $OUT/pmc_traffic.json profiles/r02/pmc_traffic.json
}
pmc cfg2 "cfg2:16777216x65536x8" "" &&
pmc cfg2cold "cfg2:16777216x65536x8:cold" "--evict" &&
pmc cfg3 "cfg3shard:134217728x131072x8" "--n 134217728 --q 131072" &&
echo pmc-ok &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 && tail -1 $OUT/bench20.log > $OUT/bench20.json &&
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log > $OUT/bench.json &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra > $OUT/kt.log 2>&1 &&
python3 tools/kt_window.py $OUT/kt 5 20 > $OUT/kt_windows.txt && python3 tools/kt_window.py $OUT/kt 25 20 >> $OUT/kt_windows.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_small -o run --output-format csv -- python3 tools/small_probe.py > $OUT/kt_small.log 2>&1 &&
DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $OUT/phase_stamps_cfg2.log 2>&1 &&
echo all-ok
