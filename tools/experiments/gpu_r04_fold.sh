# Round-4: F1 folded into F2 -- the whole GPU suite on the in-tree (folded) build, then the A/B
# against the separate-F1 build (cfg-2 1,000 / 20 steps, cfg-3 shard), then K2 occupancy variants.
set -o pipefail
OUT=gpurun_out/${1:-r04fold}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/experiments/gpu_ab_libs.sh ${1:-r04fold} none fold=tree sep=opendht_amd/ab/nofold.so || exit 1
bash tools/experiments/gpu_k2_libs.sh ${1:-r04fold}_k2 p8=tree p4=opendht_amd/ab/k2_p4.so p5=opendht_amd/ab/k2_p5.so p6=opendht_amd/ab/k2_p6.so || exit 1
echo all-ok
