# Round-3 pass C: A/B of K2 (cfg 4) and of F2's segmented ranges at the cfg-3 shard
# (DHTGPU_F2NOSEG=1: more workgroups in whole rounds instead), KS timings.
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py::test_k6_cfg2_full_batch_vs_oracle > $OUT/t0.log 2>&1 || { tail -30 $OUT/t0.log; exit 1; }
tail -1 $OUT/t0.log
timeout -k 10 120 python tools/classify_probe.py > $OUT/k2.log 2>&1 || { cat $OUT/k2.log; exit 1; }
cat $OUT/k2.log
timeout -k 10 200 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_seg.log 2>&1 || exit 1
DHTGPU_F2NOSEG=1 timeout -k 10 200 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_noseg.log 2>&1 || exit 1
grep -H "ms/call\|phases" $OUT/cfg3_*.log
timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_scale.py::test_cfg4_classify_1e8 tests/test_gpu_parity.py -k "classify or cfg4" > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for sp in 0 -1 0 -1; do
  DHTGPU_F3SPEC=$sp timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --no-cpu --no-extra --no-scan > $OUT/bench_spec$sp.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/bench_spec$sp.json')); print('spec $sp', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['kernels_ms'])"
done
export TMPDIR=/tmp
DHTGPU_F3SPEC=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/cfg3s0_fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 > $OUT/cfg3s0_fetch.log 2>&1 || exit 1
DHTGPU_F3SPEC=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/cfg2s0_fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/cfg2s0_fetch.log 2>&1 || exit 1
echo done
