set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_seg
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $O/f.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $O/w.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $O/t.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $O/tcp -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $O/p.log 2>&1 &&
python3 tools/pmc_traffic.py $O/fetch $O/write $O/traffic.json seg && echo ok
