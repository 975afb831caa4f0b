# Round-4 pass B: the whole GPU suite, the world-of-one collective bench + its kernel trace, and the
# cfg-2 / cfg-3 shard A/B of this build against opendht_amd/ab/prev.so (F4 speculative tie loads)
set -o pipefail
OUT=gpurun_out/${1:-r04b}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/experiments/gpu_r04_sharded.sh ${1:-r04b} || exit 1
bash tools/experiments/gpu_r04_kt_sharded.sh ${1:-r04b} || exit 1
bash tools/experiments/gpu_ab_libs.sh ${1:-r04b}_ab none new=tree prev=opendht_amd/ab/prev.so || exit 1
echo all-ok
