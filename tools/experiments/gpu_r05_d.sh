# Round 5, pass d: hardware queues (GPU_MAX_HW_QUEUES 4, HIP's default, against 8) for the
# world-of-one collective path and the one-GPU headline; a kernel trace of the collective path
# at 8 queues.   usage: bash tools/experiments/gpu_r05_d.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r05d}; mkdir -p $OUT
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d['latency_ms_per_batch']*1e3,1), 'enq', round(d['host_enqueue_ms_per_step']*1e3,1), 'win', round(d['gpu_window_ms_per_step']*1e3,1), 'verified', d.get('verified_exact'))"; }
for i in 1 2; do
  for hq in 4 8; do
    DHT_BENCH_HW_QUEUES=$hq timeout -k 10 300 python bench.py --sharded --steps 1000 --warmup 100 --no-cpu --no-extra --verify 16 > $OUT/sh1000_q$hq.json 2> $OUT/sh1000_q$hq.err || { tail -20 $OUT/sh1000_q$hq.err; exit 1; }
    line $OUT/sh1000_q$hq.json "sharded S=1000 hwq=$hq"
    DHT_BENCH_HW_QUEUES=$hq timeout -k 10 300 python bench.py --sharded --steps 20 --warmup 5 --no-cpu --no-extra --verify 16 > $OUT/sh20_q$hq.json 2> $OUT/sh20_q$hq.err || { tail -20 $OUT/sh20_q$hq.err; exit 1; }
    line $OUT/sh20_q$hq.json "sharded S=20 hwq=$hq"
    DHT_BENCH_HW_QUEUES=$hq timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu --no-extra --no-scan --verify 16 > $OUT/b1000_q$hq.json 2> $OUT/b1000_q$hq.err || { tail -20 $OUT/b1000_q$hq.err; exit 1; }
    line $OUT/b1000_q$hq.json "headline S=1000 hwq=$hq"
    DHT_BENCH_HW_QUEUES=$hq timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-scan --verify 16 > $OUT/b20_q$hq.json 2> $OUT/b20_q$hq.err || { tail -20 $OUT/b20_q$hq.err; exit 1; }
    line $OUT/b20_q$hq.json "headline S=20 hwq=$hq"
  done
done | tee $OUT/hwq.txt
echo all-ok
