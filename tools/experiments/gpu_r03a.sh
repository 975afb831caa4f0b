# Round-3 first pass: the new parity tests, a short bench, and F3's speculative-gather A/B
# (DHTGPU_F3SPEC: -1 plan, 0 exact gather, 512 = the round-2 fixed size) at cfg 2 and the
# cfg-3 shard, kernel times by events (tools/batch_probe.py).
set -o pipefail
OUT=gpurun_out/r03a; mkdir -p $OUT
(nproc; cat /sys/fs/cgroup/cpu.max; python -c "import os;print(len(os.sched_getaffinity(0)))"; lscpu | head -20) > $OUT/cpuinfo.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py::test_k6_cfg2_full_batch_vs_oracle tests/test_gpu_scale.py::test_index_two_threads_fresh_process tests/test_gpu_scale.py::test_cfg3_shard_2p27 > $OUT/t1.log 2>&1 || { tail -30 $OUT/t1.log; exit 1; }
tail -3 $OUT/t1.log
for sp in -1 0 512; do
  DHTGPU_F3SPEC=$sp timeout -k 10 120 python tools/batch_probe.py --reps 20 > $OUT/ab_cfg2_$sp.log 2>&1 || exit 1
  DHTGPU_F3SPEC=$sp timeout -k 10 200 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/ab_cfg3_$sp.log 2>&1 || exit 1
done
grep -H phases $OUT/ab_*.log
timeout -k 10 500 python bench.py --steps 200 --warmup 50 > $OUT/b1.json 2> $OUT/b1.err || { tail -20 $OUT/b1.err; exit 1; }
echo done
