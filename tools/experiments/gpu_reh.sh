# Multi-rank rehearsal on ONE GPU at HEAD: the N>1 headline path (2 ranks on cuda:0 over gloo,
# weak-scaled prefix route) and the N>1 cfg-3 leg (tools/rehearse_cfg3.py, a world of 1 over RCCL)
set -o pipefail
O=gpurun_out/reh; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rehearse-one-gpu --steps 100 --warmup 20 --no-cpu > $O/bench_2ranks.log 2>&1 || { tail -20 $O/bench_2ranks.log; exit 1; }
tail -1 $O/bench_2ranks.log | cut -c1-700
timeout -k 10 400 python tools/rehearse_cfg3.py > $O/rehearse_cfg3.log 2>&1 || { tail -20 $O/rehearse_cfg3.log; exit 1; }
grep -v "^\[" $O/rehearse_cfg3.log | tail -1 | cut -c1-1500
