# KS variant check (parity tests through the variant library) + S1/S2 per q A/B.
# usage: bash tools/experiments/gpu_ks_ab2.sh <out-tag> <checked-variant> <variant>...
set -o pipefail
TAG=$1; CV=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/$CV.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small_batch or fallback_scan_small" > $OUT/tests_$CV.log 2>&1 || { tail -30 $OUT/tests_$CV.log; exit 1; }
tail -1 $OUT/tests_$CV.log
bash tools/experiments/gpu_ks_ab.sh $TAG $CV "$@"
