# K3 heads merge: the merge / record / shard tests, the world-of-one collective bench (all-gather and
# all-to-all through RCCL, verified), and its kernel trace
set -o pipefail
OUT=gpurun_out/${1:-r04k3}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "merge or record or shard or scan or topk_sizes or batch_shapes" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/experiments/gpu_r04_sharded.sh ${1:-r04k3} || exit 1
bash tools/experiments/gpu_r04_kt_sharded.sh ${1:-r04k3} || exit 1
