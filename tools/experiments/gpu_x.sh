# A/B of the cfg-2 step period over the number of batches in flight (streams)
set -o pipefail
O=gpurun_out/x; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for d in 2 3 4; do
    timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan --inflight $d > $O/d${d}_$i.log 2>&1 || exit 1
    echo "d=$d $(grep timed $O/d${d}_$i.log)"
  done
done
