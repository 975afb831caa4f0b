# Round 5, pass e: where the world-of-one collective step's time goes.  Host cost of each piece
# (host_profile.py); K6 record form with F3's word-1 gather or record stores left out (DHTGPU_DBG
# 2^16 / 2^17 on the Diag build, 2^18 = the Diag build with nothing left out); the sharded bench.
# usage: bash tools/experiments/gpu_r05_e.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r05f}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/experiments/host_profile.py > $OUT/host_profile.json 2> $OUT/host_profile.err || { tail -20 $OUT/host_profile.err; exit 1; }
grep piece $OUT/host_profile.json
for d in 0 262144 65536 131072 196608; do
  DHTGPU_DBG=$d timeout -k 10 200 python tools/shard_probe.py --steps 300 > $OUT/probe_$d.json 2> $OUT/probe_$d.err || { tail -20 $OUT/probe_$d.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/probe_$d.json'):
    d = json.loads(l)
    if 'N' in d: print('dbg $d N', d['N'], 'rec', round(d['ms_per_step_records']*1e3, 1), 'idx', round(d['ms_per_step_indices']*1e3, 1), {k: round(v*1e3, 1) for k, v in d['kernels_ms_serial'].items()})
"
done
echo all-ok
