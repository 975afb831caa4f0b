# the collective path through RCCL on one GPU: bench.py --sharded (a world of one: range shard = the
# whole set, K6 record mode, RCCL all-gather / all-to-all, K3), verified against the oracle
set -o pipefail
OUT=gpurun_out/${1:-r04sh}; mkdir -p $OUT
for x in allgather alltoall; do
  timeout -k 10 300 python bench.py --sharded --exchange $x --steps 20 --warmup 5 --verify 64 > $OUT/sharded_$x.json 2> $OUT/sharded_$x.err || { tail -20 $OUT/sharded_$x.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/sharded_$x.json') if l.startswith('{')][0]); print('$x', d['config']['parallelism'], round(d['ms_per_step']*1e3,2), 'us/step lat', round(d['latency_ms_per_batch']*1e3,1), 'verified', d.get('verified_exact'), d['roofline'].get('aggregate', {}).get('traffic'))"
done
