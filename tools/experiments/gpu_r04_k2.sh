# Round-4 K2 (word-0 streaming classify): parity tests, the variants (workgroups per CU x uint4 per
# lane) three times each, PMC FETCH/WRITE of the in-tree build.   usage: bash tools/experiments/gpu_r04_k2.sh [tag]
set -o pipefail
OUT=gpurun_out/${1:-r04k2}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "classify or kat" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/experiments/gpu_k2_libs.sh ${1:-r04k2} tree=tree p8u2=opendht_amd/ab/k2_8_2.so p16u3=opendht_amd/ab/k2_16_3.so p4u3=opendht_amd/ab/k2_4_3.so p16u1=opendht_amd/ab/k2_16_1.so p12u3=opendht_amd/ab/k2_12_3.so || exit 1
cp profiles/r04/pmc_traffic.json $OUT/pmc_traffic.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/k2_fetch -o run --output-format csv -- python3 tools/classify_probe.py --reps 3 > $OUT/k2_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/k2_write -o run --output-format csv -- python3 tools/classify_probe.py --reps 3 > $OUT/k2_write.log 2>&1 &&
python3 tools/pmc_traffic.py $OUT/k2_fetch $OUT/k2_write $OUT/pmc_traffic.json "cfg4:100000000" | grep -A4 k_classify || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_k2 -o run --output-format csv -- python3 tools/classify_probe.py --reps 20 > $OUT/kt_k2.log 2>&1 || exit 1
grep -h "k_classify" $OUT/kt_k2/*stats* | head -3
echo all-ok
